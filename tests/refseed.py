"""TEST INFRASTRUCTURE ONLY — ChainsRecords seeded by the REFERENCE itself.

Runs oracle/_ref/gen_golden (the reference's own bwa C built by oracle/Makefile:
bwa index of the synthetic 1 Mb golden genome with repeats / N runs / contig
junctions, then mem_chain -> mem_chain_flt -> mem_flt_chained_seeds per read,
then the reference mem_chain2aln, see oracle/gen_golden.c) into a scratch
directory and loads the result: the batch exactly as bwa-flow's SeqsToChains
stage hands it to ChainsToRegions (src/Pipeline.cpp:503-544), the reference's
regions for it, and the reference genome.

Used by the C2-sized `-m gpu` parity test and tools_dev/realbench.py: a batch
of 33,334 pairs (66,668 reads, >= 10 Mbases — one ChainsRecord,
Pipeline.cpp:123,146) takes ~5 s to make on one host core.
"""
from __future__ import annotations

import os
import subprocess
import tempfile

import numpy as np

from bwagpu import abi
from bwagpu.engine import Batch

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
GEN = os.path.join(REPO, "oracle", "_ref", "gen_golden")
OPT_KEYS = ("a", "b", "o_del", "e_del", "o_ins", "e_ins", "pen_clip5", "pen_clip3", "w", "zdrop")


def available() -> bool:
    return os.access(GEN, os.X_OK)


def _rd(d, name, dt):
    return np.fromfile(os.path.join(d, name + ".bin"), dtype=dt)


def load_dump(d: str):
    """-> opt, ref dict, Batch, expected regions (compact, read order), expected counts"""
    oi = _rd(d, "opt_int", np.int32)
    opt = dict(zip(OPT_KEYS, oi.tolist()))
    opt["mat"] = _rd(d, "opt_mat", np.int8)
    ref = dict(l_pac=int(_rd(d, "l_pac", np.int64)[0]), ann_offset=_rd(d, "ann_offset", np.int64),
               ann_len=_rd(d, "ann_len", np.int32), pac=_rd(d, "pac", np.uint8))
    b = Batch(_rd(d, "seq_off", np.int64), _rd(d, "seq", np.uint8), _rd(d, "read_chain_off", np.int32),
              _rd(d, "chain_seed_off", np.int32), _rd(d, "chain_rid", np.int32),
              _rd(d, "chain_frac_rep", np.float32), _rd(d, "seeds", abi.SEED_DTYPE))
    regs = _rd(d, "regs", abi.ALNREG_DTYPE)
    n = _rd(d, "reg_n", np.int32)
    return opt, ref, b, regs, n


def make(pairs: int = 33334, seed: int = 7, length: str = "150", opt_mode: int = 0, workdir: str | None = None):
    """generate with the reference and load; length: "150" | "100" | "250" | "mix" """
    if not available():
        raise FileNotFoundError(f"{GEN} not built (make -C oracle ref, needs /root/reference)")
    own = workdir is None
    d = tempfile.mkdtemp(prefix="refseed_") if own else workdir
    os.makedirs(d, exist_ok=True)
    subprocess.run([GEN, d, str(seed), str(pairs), length, str(opt_mode)], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    out = load_dump(d)
    if own:
        for f in os.listdir(d):
            os.unlink(os.path.join(d, f))
        os.rmdir(d)
    return out
