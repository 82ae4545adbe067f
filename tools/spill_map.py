#!/usr/bin/env python3
"""Where a kernel's scratch (spill) accesses sit relative to its barriers and
the gather asm (s_set_gpr_idx_on): `python3 tools/spill_map.py k.s k_fused`."""
import re
import sys


def main(path, pat):
    s = open(path).read()
    names = [m.group(1) for m in re.finditer(r'^(\S*' + pat + r'\S*):', s, re.M)]
    for name in names[:1]:
        i = s.index(name + ':')
        j = s.index('.Lfunc_end', i)
        body = s[i:j].split('\n')
        marks = []
        for n, l in enumerate(body):
            t = l.strip()
            if t.startswith('scratch_'):
                marks.append((n, 'SPILL ' + t.split(';')[0][:60]))
            elif t.startswith('s_barrier'):
                marks.append((n, 'barrier'))
            elif 's_set_gpr_idx_on' in t:
                marks.append((n, 'gather'))
            elif t.startswith('s_cbranch') or t.startswith('s_branch'):
                marks.append((n, t[:40]))
            elif re.match(r'\.LBB\d+_\d+:', t):
                marks.append((n, t))
        prev = None
        for n, m in marks:
            if m == 'gather' and prev == 'gather':
                continue
            print(n, m)
            prev = m


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
