G = [list(range(0,4))+list(range(12,16))+list(range(20,28)),
     list(range(4,12))+list(range(16,20))+list(range(28,32)),
     list(range(32,36))+list(range(44,48))+list(range(52,60)),
     list(range(36,44))+list(range(48,52))+list(range(60,64))]
def ok(Xf, PR, PC, PG):
    for row in range(PR):
        for pg in range(PG):
            for so in (0, 1, 2):
                for c in (0, 1):
                    for grp in G:
                        seen=set()
                        for l in grp:
                            li, g = l & 15, l >> 4
                            img, col = li >> 2, li & 3
                            slot = 4*pg + so + col
                            P = (img*PR + row)*PC + slot
                            pos = (4*c + g) ^ Xf(img, row, slot)
                            u = (8*(P & 1) + pos) & 15
                            if u in seen: return False
                            seen.add(u)
    return True
pswz = lambda img, row, slot: 2*(slot & 3)
for cfg in [(4,10,2),(4,18,4),(6,18,4),(6,10,2),(10,10,2),(4,6,1),(6,6,1),(10,6,1),(12,6,1)]:
    print(cfg, ok(pswz, *cfg))
import itertools
def bits(img, row, slot):
    return [img & 1, (img >> 1) & 1, slot & 1, (slot >> 1) & 1, (slot >> 2) & 1, row & 1]
configs=[(4,10,2),(4,18,4),(6,18,4),(6,10,2),(10,10,2),(4,6,1),(6,6,1),(10,6,1)]
found=[]
for cols in itertools.product(range(8), repeat=6):
    def Xf(img, row, slot, cols=cols):
        x=0
        for b_, m in zip(bits(img,row,slot), cols):
            if b_: x ^= m
        return x
    if all(ok(Xf, *c) for c in configs):
        found.append(cols)
        if len(found) > 8: break
print(found)
