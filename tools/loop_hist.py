"""Instruction histogram of the antenna loop of a trial_kernel assembly dump (tools/one_inst.hip -S)."""
import collections
import re
import sys

L = open(sys.argv[1]).read().split('\n')
# the largest loop: header label with the most "in Loop: Header=<it>" blocks
hdrs = collections.Counter(m.group(1) for l in L for m in [re.search(r'Header=(BB\d+_\d+) Depth=1', l)] if m)


def body(h):
    out, inblk = [], False
    for l in L:
        if re.match(r'^\.LBB\d+_\d+:', l):
            inblk = ('Header=' + h) in l or l.startswith('.L' + h + ':')
            continue
        s = l.strip()
        if inblk and s and s[0] not in ';.':
            out.append(s.split()[0])
    return out


sizes = {h: body(h) for h in hdrs}
for h, b in sizes.items():
    print('  loop', h, len(b), 'instrs,', b.count('v_mad_u64_u32'), 'v_mad_u64_u32')
# default: the loop with the most Philox products (the array pass)
hdr = sys.argv[3] if len(sys.argv) > 3 else max(sizes, key=lambda h: (sizes[h].count('v_mad_u64_u32'), len(sizes[h])))
c = collections.Counter()
inblk = False
for l in L:
    if re.match(r'^\.LBB\d+_\d+:', l):
        inblk = ('Header=' + hdr) in l or l.startswith('.L' + hdr + ':')
        continue
    if not inblk:
        continue
    s = l.strip()
    if not s or s[0] in ';.':
        continue
    c[s.split()[0]] += 1
print('loop', hdr, 'total', sum(c.values()))
cls = collections.Counter()
for op, n in c.items():
    if op.startswith('v_pk_'): k = 'valu_pk'
    elif op.startswith(('v_log', 'v_exp', 'v_sin', 'v_cos', 'v_rsq', 'v_sqrt', 'v_rcp')): k = 'trans'
    elif re.match(r'v_(fma|mul|add|sub|fmac|fmamk|fmaak|max|min|ldexp|frexp|floor|fract)\w*_f32', op): k = 'valu_f32'
    elif op.startswith('v_mov'): k = 'mov'
    elif op.startswith('v_cndmask') or op.startswith('v_cmp'): k = 'cmp/cnd'
    elif op.startswith('v_'): k = 'valu_int/other'
    elif op.startswith('ds_'): k = 'lds'
    elif op.startswith(('global_', 'flat_', 'buffer_')): k = 'vmem'
    elif op.startswith('s_nop'): k = 's_nop'
    elif op.startswith('s_'): k = 'salu/branch'
    else: k = 'other'
    cls[k] += n
for k, n in cls.most_common(): print(f'  {k:16s}{n}')
for op, n in c.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 30): print(f'{op:28s}{n}')
