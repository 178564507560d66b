#!/usr/bin/env python3
"""Memory/LDS/barrier skeleton of one kernel in a hipcc -S listing (no GPU):
   python tools/isa_skel.py FILE.s NAME_SUBSTRING [max_lines]"""
import re
import sys

s = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2]
mx = int(sys.argv[3]) if len(sys.argv) > 3 else 400
start = next(i for i, l in enumerate(s) if re.match(r'^_Z\S*' + re.escape(pat) + r'\S*:', l))
end = next(i for i in range(start, len(s)) if s[i].startswith('.Lfunc_end'))
keep = re.compile(r'(buffer_load|global_load|s_waitcnt|s_barrier|ds_\w+|global_store|buffer_store|global_atomic|s_cbranch|s_branch|\.LBB|scratch_)')
n = 0
for i in range(start, end):
    t = s[i].strip()
    if keep.match(t):
        print(f'{i - start:5d}: {t[:110]}')
        n += 1
        if n >= mx:
            break
