"""ctypes wrapper of lib/libsynth.so: seeded synthetic references, read pairs
and their chains in the shape of BASELINE.json's configs (see tools/synth.cpp).
Input generation only — never part of the measured path."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import abi
from .engine import Batch, _ptr

_lib = None


def _load():
    global _lib
    if _lib is None:
        p = os.path.join(abi.LIB_DIR, "libsynth.so")
        if not os.path.exists(p):
            raise RuntimeError(f"{p} missing: run __graft_entry__.build()")
        lib = C.CDLL(p)
        lib.synth_ref.argtypes = [C.c_uint64, C.c_int64, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.synth_ref.restype = C.c_int
        lib.synth_bounds.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.synth_reads.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int, C.c_uint64, C.c_int,
                                    C.c_int, C.c_int] + [C.c_void_p] * 10
        lib.synth_reads.restype = C.c_int
        _lib = lib
    return _lib


class SynthRef:
    def __init__(self, seed: int, length: int, n_ctg: int):
        lib = _load()
        self.l_pac = int(length)
        self.pac = np.zeros(self.l_pac // 4 + 1, np.uint8)
        self.ann_offset = np.zeros(n_ctg, np.int64)
        self.ann_len = np.zeros(n_ctg, np.int32)
        rc = lib.synth_ref(seed, self.l_pac, n_ctg, _ptr(self.pac), _ptr(self.ann_offset), _ptr(self.ann_len))
        if rc:
            raise RuntimeError("synth_ref failed")


def synth_batch(ref: SynthRef, seed: int, n_pairs: int, len_mode: int = 150, min_seed_len: int = 19) -> Batch:
    """len_mode 100/150/250, or 0 for equal thirds of 100/150/250"""
    lib = _load()
    ms, mc, mseed = C.c_int64(), C.c_int32(), C.c_int32()
    lib.synth_bounds(n_pairs, len_mode, C.byref(ms), C.byref(mc), C.byref(mseed))
    nr_max = 2 * n_pairs
    seq_off = np.zeros(nr_max + 1, np.int64)
    seq = np.zeros(ms.value, np.uint8)
    rco = np.zeros(nr_max + 1, np.int32)
    cso = np.zeros(mc.value + 1, np.int32)
    rid = np.zeros(mc.value, np.int32)
    fr = np.zeros(mc.value, np.float32)
    seeds = np.zeros(mseed.value, abi.SEED_DTYPE)
    nr, nc, ns = C.c_int32(), C.c_int32(), C.c_int32()
    rc = lib.synth_reads(_ptr(ref.pac), ref.l_pac, _ptr(ref.ann_offset), _ptr(ref.ann_len), len(ref.ann_len), seed,
                         n_pairs, len_mode, min_seed_len, _ptr(seq_off), _ptr(seq), _ptr(rco), _ptr(cso), _ptr(rid),
                         _ptr(fr), _ptr(seeds), C.byref(nr), C.byref(nc), C.byref(ns))
    if rc:
        raise RuntimeError("synth_reads failed")
    r, c, s = nr.value, nc.value, ns.value
    return Batch(seq_off[:r + 1], seq[:seq_off[r]], rco[:r + 1], cso[:c + 1], rid[:c], fr[:c], seeds[:s])
