import itertools
G = [list(range(0,4))+list(range(12,16))+list(range(20,28)),
     list(range(4,12))+list(range(16,20))+list(range(28,32)),
     list(range(32,36))+list(range(44,48))+list(range(52,60)),
     list(range(36,44))+list(range(48,52))+list(range(60,64))]
def ok(X):
    for h in (0,1):
        for grp in G:
            seen=set()
            for l in grp:
                li, g = l & 15, l >> 4
                P = li
                u = 8*(P & 1) + (((4*h+g) ^ X(P)) & 7)
                if u in seen: return False
                seen.add(u)
    return True
res=[]
for cols in itertools.product(range(8), repeat=4):
    X=lambda P, cols=cols: (cols[0] if P&1 else 0) ^ (cols[1] if P&2 else 0) ^ (cols[2] if P&4 else 0) ^ (cols[3] if P&8 else 0)
    if ok(X): res.append(cols)
print(len(res), res[:10])
