"""Child process of tests/test_gpu_variants.py: the C2 fixture's two batches
and the C5 fixture's batch through bwagpu_chain2aln (host buffers) under the
BWAGPU_* knobs its environment sets (the library reads them once per
process), each checked byte for byte against the reference's regions.
Prints one JSON line."""
import json
import os
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bwa-flow_amd", "python"))
from bwagpu import workload  # noqa: E402
from bwagpu.engine import Engine  # noqa: E402


def main():
    out = {}
    opt, ref, rbs = workload.load_fixture()
    eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
    out["c2"] = [bool(rb.check(*eng.chain2aln(rb.batch))) for rb in rbs]
    eng.close()
    opt5, _, rbs5 = workload.load_fixture(workload.C5_FIXTURE, with_ref=False)
    eng = Engine(0, opt5, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
    out["c5"] = [bool(rb.check(*eng.chain2aln(rb.batch))) for rb in rbs5]
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
