import sys, os
sys.path.insert(0, 'bwa-flow_amd/python'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
import numpy as np
import golden_io as G, oracle
from bwagpu.engine import Engine
refd = G.load_ref()
for name in G.CHAIN_SETS + G.KSW_SETS:
    opt, tasks, want, qp, tp = G.load_tasks(name)
    eng = Engine(0, opt, refd["l_pac"], refd["ann_offset"], refd["ann_len"], pac=refd["pac"])
    got = eng.extend_batch(tasks, qp, tp)
    g, w = got.view(np.int32).reshape(-1, 6), want.view(np.int32).reshape(-1, 6)
    bad = np.nonzero((g != w).any(axis=1))[0]
    print(name, "bad", len(bad), "of", len(tasks))
    for i in bad[:6]:
        print("  task", tasks[i], "got", g[i], "want", w[i])
    eng.close()
