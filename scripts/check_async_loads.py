# Dev check: in the register-streamed 1x1 kernels (csrc/conv_rs.hip) X is loaded by inline asm, so hipcc
# does not know the registers are written asynchronously; flag any instruction that reads a loaded
# register before the next s_waitcnt vmcnt (usage: check_async_loads.py <hipcc --save-temps .s file>).
import re, sys
s = open(sys.argv[1]).read()
def regs_of(txt):
    out = set()
    for a, b in re.findall(r'v\[(\d+):(\d+)\]', txt):
        out.update(range(int(a), int(b) + 1))
    for x in re.findall(r'(?<![\w\[:])v(\d+)\b', txt):
        out.add(int(x))
    return out
for m in re.finditer(r'^(_ZN3yv712_GLOBAL__N_117conv1x1_rs_kernel(\S+?)EEEvNS\S+):.*?\.Lfunc_end', s, re.S | re.M):
    name = m.group(2)
    lines = [l.strip() for l in m.group(0).split('\n')]
    bad = []
    for i, l in enumerate(lines):
        mm = re.match(r'buffer_load_dwordx4 v\[(\d+):(\d+)\]', l)
        if not mm:
            continue
        live = set(range(int(mm.group(1)), int(mm.group(2)) + 1))
        for l2 in lines[i + 1:]:
            if l2.startswith('s_waitcnt') and 'vmcnt' in l2:
                break
            if not l2 or l2.startswith(';') or l2.startswith('.'):
                continue
            op = l2.split()[0]
            rest = l2[len(op):]
            if op.startswith('buffer_store') or op.startswith('s_') or op.startswith('ds_write'):
                srcs = regs_of(rest)
                dst = set()
            else:
                parts = rest.split(',', 1)
                dst = regs_of(parts[0])
                srcs = regs_of(parts[1]) if len(parts) > 1 else set()
                if op.startswith('buffer_load'):
                    srcs = regs_of(parts[1].split(',')[0]) if len(parts) > 1 else set()
            if srcs & live:
                bad.append((l, l2))
                break
            live -= dst
            if not live:
                break
    print(name, 'early reads of in-flight X registers:', len(bad), bad[:2])
