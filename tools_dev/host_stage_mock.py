#!/usr/bin/env python3
"""The drop-in stage's host side with the device taken out (development tool):
bench.py's end_to_end leg (host/stage_bench.cpp gpustage_run) linked against
tools_dev/micro/host_stage_mock.cpp instead of libbwagpu.so, so every record's
'device' work is free and what remains is ChainsToRegionsGPU's host work
(pack, malloc'd mem_alnreg_v, chain frees, the sink).  Runs on the CPU.

    python tools_dev/host_stage_mock.py [workers] [reps] [chain_mode] [sink_workers]
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bwa-flow_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
from bwagpu import abi, workload  # noqa: E402
from bwagpu.engine import compact  # noqa: E402
import oracle  # noqa: E402

SO = os.path.join(REPO, "tools_dev", "micro", "libgpustage_mock.so")


def build():
    src = [os.path.join(REPO, "tools_dev", "micro", "host_stage_mock.cpp"),
           os.path.join(REPO, "bwa-flow_amd", "host", "stage_bench.cpp"),
           os.path.join(REPO, "bwa-flow_amd", "host", "GPUPipeline.cpp")]
    subprocess.run(["g++", "-O2", "-g", "-fPIC", "-shared", "-std=c++17", "-I" + os.path.join(REPO, "include"),
                    "-I" + os.path.join(REPO, "bwa-flow_amd", "host"), "-I/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", *src, "-o", SO, "-lpthread"], check=True)


def main():
    workers = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    chain_mode = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    sink = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    build()
    lib = C.CDLL(SO)
    opt, ref, rbs = workload.load_fixture()
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    batches = [rb.batch for rb in rbs]
    for b in batches:
        regs, n, _ = oracle.chain2aln("ref", opt, R, b, n_threads=8)
        c = np.ascontiguousarray(compact(b, regs, n))
        lib.mock_register(b.n_reads, b.n_chains, b.n_seeds, c.ctypes.data_as(C.c_void_p),
                          np.ascontiguousarray(n, np.int32).ctypes.data_as(C.c_void_p))
    lib.gpustage_run.restype = C.c_int
    o = abi.opt_from_dict(opt)
    bns = abi.Bns()
    bns.l_pac, bns.n_seqs = ref.l_pac, len(ref.ann_len)
    ann_off = np.ascontiguousarray(ref.ann_offset, np.int64)
    ann_len = np.ascontiguousarray(ref.ann_len, np.int32)
    bns.ann_offset = ann_off.ctypes.data_as(C.c_void_p)
    bns.ann_len = ann_len.ctypes.data_as(C.c_void_p)
    pac = np.ascontiguousarray(ref.pac, np.uint8)
    arr = (abi.BatchC * len(batches))(*[b.to_c() for b in batches])
    outs_n = [np.zeros(b.n_reads, np.int32) for b in batches]
    outs_r = [np.zeros(b.n_seeds, abi.ALNREG_DTYPE) for b in batches]
    pn = (C.c_void_p * len(batches))(*[x.ctypes.data for x in outs_n])
    pr = (C.c_void_p * len(batches))(*[x.ctypes.data for x in outs_r])
    times = np.zeros(12, np.float64)
    rc = lib.gpustage_run(C.byref(o), C.byref(bns), pac.ctypes.data_as(C.c_void_p), len(batches), arr, reps, 1,
                          workers, chain_mode, sink, times.ctypes.data_as(C.c_void_p), C.cast(pn, C.c_void_p),
                          C.cast(pr, C.c_void_p))
    nrec = max(int(times[5]), 1)
    ok = all(rb.check_compact(r, n) for rb, r, n in zip(rbs, outs_r, outs_n))
    reads = reps * sum(b.n_reads for b in batches)
    print(f"rc={rc} workers={workers} chain_mode={chain_mode} sink={sink} records={nrec} "
          f"value={reads / times[0] / 1e6:.2f} Mreads/s wall={times[0] * 1e3 / nrec:.3f} ms/record  per record "
          + " ".join(f"{k}={v * 1e3 / nrec:.3f}" for k, v in zip(("pack", "submit", "wait", "post"), times[1:5]))
          + f" cpu_ms_per_record user={times[10] * 1e3 / nrec:.2f} sys={times[11] * 1e3 / nrec:.2f}"
          + f" parity={ok} cpus={os.cpu_count()}")


if __name__ == "__main__":
    main()
