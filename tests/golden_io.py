"""Loaders for the committed golden vectors in tests/golden/ (made by
oracle/gen_golden.py from the reference's own C; see its docstring)."""
from __future__ import annotations

import os

import numpy as np

from bwagpu import abi
from bwagpu.engine import Batch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CHAIN_SETS = ["c1_default", "c5_mixed", "opt1_scoring", "opt2_band"]
KSW_SETS = ["ksw_edge_default", "ksw_edge_scoring", "ksw_edge_matrix"]
ALIGN2_SETS = ["align2_default", "align2_scoring", "align2_cheapgap", "align2_cheapdel"]
OPT_KEYS = ("a", "b", "o_del", "e_del", "o_ins", "e_ins", "pen_clip5", "pen_clip3", "w", "zdrop")


def _npz(name):
    return np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)


def load_ref():
    z = _npz("ref")
    return dict(l_pac=int(z["l_pac"][0]), ann_offset=z["ann_offset"], ann_len=z["ann_len"], pac=z["pac"])


def opt_of(z) -> dict:
    o = dict(zip(OPT_KEYS, z["opt_int"].tolist()))
    o["mat"] = z["opt_mat"].astype(np.int8)
    return o


def load_chain_set(name):
    """-> opt, Batch, expected regions (read order, compact), expected per-read counts"""
    z = _npz(name)
    b = Batch(z["seq_off"], z["seq"], z["read_chain_off"], z["chain_seed_off"], z["chain_rid"],
              z["chain_frac_rep"], z["seeds"])
    return opt_of(z), b, z["regs"].astype(abi.ALNREG_DTYPE), z["reg_n"]


def load_tasks(name):
    """-> opt, tasks, expected results, qpool, tpool"""
    z = _npz(name)
    return opt_of(z), z["tasks"].astype(abi.EXT_TASK_DTYPE), z["task_res"].astype(abi.EXT_RES_DTYPE), \
        z["qpool"], z["tpool"]


def load_align2(name):
    """ksw_align2 set -> opt, tasks, expected kswr_t records, qpool, tpool"""
    z = _npz(name)
    return opt_of(z), z["tasks"].astype(abi.ALIGN2_TASK_DTYPE), z["task_res"].astype(abi.KSWR_DTYPE), \
        z["qpool"], z["tpool"]


def kswr_mismatch(tasks, got, want) -> str | None:
    g, w = got.view(np.int32).reshape(-1, 7), want.view(np.int32).reshape(-1, 7)
    bad = np.nonzero((g != w).any(axis=1))[0]
    if len(bad) == 0:
        return None
    i = int(bad[0])
    return f"{len(bad)}/{len(tasks)} tasks differ; first #{i} {tasks[i]}: got {got[i]} want {want[i]}"


def region_mismatch(got: np.ndarray, want: np.ndarray) -> str | None:
    """bit-exact comparison of mem_alnreg_t arrays; a readable diff or None"""
    if len(got) != len(want):
        return f"region count {len(got)} != {len(want)}"
    g = got.view(np.uint8).reshape(len(got), 88) if len(got) else np.zeros((0, 88), np.uint8)
    w = want.view(np.uint8).reshape(len(want), 88) if len(want) else np.zeros((0, 88), np.uint8)
    bad = np.nonzero((g != w).any(axis=1))[0]
    if len(bad) == 0:
        return None
    i = int(bad[0])
    fields = [f for f in abi.ALNREG_DTYPE.names if got[i][f] != want[i][f]]
    return (f"{len(bad)} regions differ; first #{i}: fields {fields}: "
            f"got {[got[i][f] for f in fields]} want {[want[i][f] for f in fields]}")
