"""Per-basic-block instruction counts of one loop of a trial_kernel assembly dump.

usage: python tools/loop_blocks.py <dump.s> <loop header, e.g. BB0_57>
Shows which blocks of the antenna loop hold the Philox products, transcendentals,
barriers and LDS traffic, so the executed path (one PA kind, one channel) can be told
apart from the statically compiled-in alternatives.
"""
import collections
import re
import sys

KEYS = ('v_mad_u64_u32', 'v_exp_f32_e32', 'v_log_f32_e32', 'v_rsq_f32_e32', 'v_sqrt_f32_e32', 'v_sin_f32_e32',
        's_barrier', 'ds_write2_b64', 'ds_read2_b64', 's_nop', 'v_mov_b32_e32', 'v_cndmask_b32_e32',
        'global_load_dwordx2')


def main():
    lines = open(sys.argv[1]).read().split('\n')
    hdr = sys.argv[2]
    blocks, cur = [], None
    for line in lines:
        m = re.match(r'^\.L(BB\d+_\d+):(.*)', line)
        if m:
            cur = [m.group(1), m.group(2).strip(), collections.Counter()]
            blocks.append(cur)
            continue
        s = line.strip()
        if cur and s and s[0] not in ';.':
            cur[2][s.split()[0]] += 1
    for name, comment, c in blocks:
        if name == hdr or ('Header=' + hdr) in comment:
            key = {k: c[k] for k in KEYS if c[k]}
            print(name, sum(c.values()), key)


if __name__ == '__main__':
    main()
