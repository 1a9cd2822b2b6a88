"""Print the instruction-class sequence of the main K loop of kernels in a hipcc -S file.
M = MFMA, G = LDS-DMA (global_load_lds), D = ds_read, W = ds_write, | = s_barrier,
v<n> = s_waitcnt vmcnt(n), l<n> = lgkmcnt(n), b = branch.  Usage: asm_loop.py file.s name_fragment"""
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
frag = sys.argv[2]
for i, l in enumerate(lines):
    m = re.match(r'^(_Z\S+):', l)
    if not m or frag not in m.group(1):
        continue
    end = next(j for j in range(i, len(lines)) if lines[j].strip().startswith('s_endpgm'))
    vg = [x for x in lines[end:end + 400] if 'num_vgpr' in x and m.group(1) in x]
    seq = []
    for x in lines[i:end]:
        x = x.strip()
        if x.startswith('s_waitcnt'):
            w = re.findall(r'(vmcnt|lgkmcnt)\((\d+)\)', x)
            seq.append(''.join(('v' if a == 'vmcnt' else 'l') + b for a, b in w) + ' ')
            continue
        for pre, c in (('v_mfma', 'M'), ('global_load_lds', 'G'), ('ds_read', 'D'), ('ds_write', 'W'),
                       ('s_barrier', '|'), ('s_cbranch', 'b')):
            if x.startswith(pre):
                seq.append(c)
    s = ''.join(seq)
    best = max(s.split('|'), key=lambda x: x.count('M'))
    print(m.group(1), vg[0].split(',')[-1].strip() if vg else '')
    print('  ', best)
