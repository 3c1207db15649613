#!/usr/bin/env python3
"""Which state left by the bench's headline leg slows the GRCh38 regime leg
(c3_refseed: 2.56 ms per batch inside bench.py, 1.75-1.80 in a fresh process).

Runs the headline's set-up (C2 engine, both batches resident with 30 output
sets, torch's current stream set to the launch stream, 30 steps on 2 streams),
then times c3_refseed (tools_dev/regime_ab.py's pattern) after each release:

    live      headline engine + batches alive, current stream set
    nostream  torch's current stream back to the default
    closed    headline engine closed
    freed     headline batches freed, caching allocator emptied
"""
import json
import os
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "bwa-flow_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tools_dev"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import regime_ab  # noqa: E402
from bwagpu import workload  # noqa: E402
from bwagpu.engine import Engine  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    opt, gref, rbs = workload.load_fixture(with_ref=True)
    pac_t = torch.from_numpy(gref.pac).to(dev)
    eng = Engine(0, opt, gref.l_pac, gref.ann_offset, gref.ann_len, pac_device_ptr=pac_t.data_ptr())
    eng.set_device_read_len(max(int(np.diff(rb.batch.seq_off).max()) for rb in rbs))
    dbs = [bench.DevBatch(rb.batch, dev, rb) for rb in rbs]
    for i in range(2, 30):
        dbs[i % 2].add_out()
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    streams = [stream, torch.cuda.Stream(device=dev)]
    for i in range(30):
        dbs[i % 2].run(eng, streams[i % 2].cuda_stream, i // 2)
    torch.cuda.synchronize()

    opt3, g2, s = workload.load_c3_refseed()
    pac3 = torch.from_numpy(g2.pac).to(dev)
    regime_ab.STREAMS.extend(torch.cuda.Stream(device=dev) for _ in range(2))
    out = {}

    def c3r(tag):
        e3 = Engine(0, opt3, g2.l_pac, g2.ann_offset, g2.ann_len, pac_device_ptr=pac3.data_ptr())
        e3.set_device_read_len(int(np.diff(s.batch.seq_off).max()))
        d = [(bench.DevBatch(s.batch, dev), lambda r, n: s.check(r, n) is None)]
        out[tag] = regime_ab.timed(e3, d, [0], 2, 10, stats=True, prof=True)
        print(tag, out[tag], file=sys.stderr, flush=True)
        e3.close()

    c3r("live")
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    c3r("nostream")
    eng.close()
    c3r("closed")
    del dbs
    torch.cuda.empty_cache()
    c3r("freed")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
