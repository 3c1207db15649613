#!/usr/bin/env python3
"""Instruction mix of the innermost loops of kernels in a gfx950 .s file.
    python tools_dev/loopstat.py file.s kernel_substring [min_len]"""
import re, sys
s = open(sys.argv[1]).read()
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 100
for m in re.finditer(r'^(_Z\S*' + re.escape(sys.argv[2]) + r'\S*):', s, re.M):
    name = m.group(1); i = m.start(); j = s.index('.Lfunc_end', i)
    body = s[i:j].split('\n')
    labels = {}
    for k, l in enumerate(body):
        mm = re.match(r'^(\.LBB\w+):', l)
        if mm: labels[mm.group(1)] = k
    for k, l in enumerate(body):
        mm = re.search(r's_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)', l)
        if not mm: continue
        t = mm.group(1) or mm.group(2)
        if t in labels and labels[t] < k:
            seg = body[labels[t]:k + 1]
            ins = [x.strip() for x in seg if x.strip() and not x.strip().startswith(('.', ';', '//')) and ':' not in x.split()[0]]
            if len(ins) < minlen or len(ins) > 600: continue
            v = sum(1 for x in ins if x.startswith('v_'))
            sa = sum(1 for x in ins if x.startswith('s_') and not x.startswith(('s_nop', 's_waitcnt')))
            nop = sum(1 for x in ins if x.startswith('s_nop'))
            dpp = sum(1 for x in ins if '_dpp' in x)
            w = sum(1 for x in ins if x.startswith('s_waitcnt'))
            print(f"{name[:60]:60s} {t:10s} len {len(ins):4d} valu {v:4d} dpp {dpp:3d} salu {sa:3d} nop {nop:3d} wait {w}")
