"""Dumps the C2 batch 0 arrays for tools_dev/micro/check_scan (argv[1]: out dir)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "bwa-flow_amd", "python"))
import numpy as np  # noqa: E402

from bwagpu import workload  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
b = workload.load_fixture()[2][0].batch
for f in ("seq_off", "read_chain_off", "chain_seed_off", "seeds"):
    np.ascontiguousarray(getattr(b, f)).tofile(os.path.join(out, f + ".bin"))
