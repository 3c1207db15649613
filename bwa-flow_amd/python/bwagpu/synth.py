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
        lib.golden_genome.argtypes = [C.c_uint64, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.golden_genome.restype = C.c_int
        lib.synth_reads_genome.argtypes = lib.synth_reads.argtypes
        lib.synth_reads_genome.restype = C.c_int
        lib.grch38_layout.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        lib.grch38_layout.restype = C.c_int
        lib.grch38_genome.argtypes = [C.c_uint64, C.c_void_p, C.c_int]
        lib.grch38_genome.restype = C.c_int
        _lib = lib
    return _lib


class GoldenRef:
    """the genome of the reference-seeded workloads (tools/synth.cpp
    golden_genome = oracle/gen_golden.c's generator + bwa's N filling): the
    pac bwa_idx_build makes of it, three contigs"""

    def __init__(self, length: int, seed: int = 1234):
        lib = _load()
        self.l_pac = int(length)
        self.pac = np.zeros(self.l_pac // 4 + 1, np.uint8)
        self.ann_offset = np.zeros(3, np.int64)
        self.ann_len = np.zeros(3, np.int32)
        if lib.golden_genome(seed, self.l_pac, _ptr(self.pac), _ptr(self.ann_offset), _ptr(self.ann_len)):
            raise RuntimeError("golden_genome failed")


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


class Grch38Ref:
    """the C3 regime's reference (tools/synth.cpp grch38_layout/grch38_genome):
    GRCh38's 195-contig table and l_pac (3,099,734,149), seeded content; the
    pac is 0.78 GB"""

    N_CTG = 195

    def __init__(self, seed: int = 38, threads: int | None = None):
        lib = _load()
        self.ann_offset = np.zeros(self.N_CTG, np.int64)
        self.ann_len = np.zeros(self.N_CTG, np.int32)
        lp = C.c_int64()
        if lib.grch38_layout(_ptr(self.ann_offset), _ptr(self.ann_len), C.byref(lp)) != self.N_CTG:
            raise RuntimeError("grch38_layout failed")
        self.l_pac = int(lp.value)
        self.pac = np.empty(self.l_pac // 4 + 1, np.uint8)
        nt = threads or min(16, os.cpu_count() or 1)
        if lib.grch38_genome(seed, _ptr(self.pac), nt):
            raise RuntimeError("grch38_genome failed")


def synth_batch(ref, seed: int, n_pairs: int, len_mode: int = 150, min_seed_len: int = 19,
                genome_wide: bool = False) -> Batch:
    """len_mode 100/150/250, or 0 for equal thirds of 100/150/250; genome_wide:
    C3 placement (contigs weighted by length, one pair in ten across a contig
    junction) instead of a uniform contig"""
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
    fn = lib.synth_reads_genome if genome_wide else lib.synth_reads
    rc = fn(_ptr(ref.pac), ref.l_pac, _ptr(ref.ann_offset), _ptr(ref.ann_len), len(ref.ann_len), seed,
            n_pairs, len_mode, min_seed_len, _ptr(seq_off), _ptr(seq), _ptr(rco), _ptr(cso), _ptr(rid),
            _ptr(fr), _ptr(seeds), C.byref(nr), C.byref(nc), C.byref(ns))
    if rc:
        raise RuntimeError("synth_reads failed")
    r, c, s = nr.value, nc.value, ns.value
    return Batch(seq_off[:r + 1], seq[:seq_off[r]], rco[:r + 1], cso[:c + 1], rid[:c], fr[:c], seeds[:s])


def _mutate(rng, q, sub=0.03, indel=0.01):
    """a diverged copy of q: substitutions, 1-3 base indels, N kept as N"""
    out = []
    r = rng.random(len(q))
    for k, b in enumerate(q.tolist()):
        x = r[k]
        if x < indel / 2:
            continue
        if x < indel:
            out.extend(rng.integers(0, 4, int(rng.integers(1, 4))).tolist())
        out.append(int(rng.integers(0, 4)) if (b < 4 and rng.random() < sub) else b)
    return np.array(out, np.uint8)


def mate_rescue_tasks(rng, n, a=1, min_seed_len=19, qlens=(150,), win=(300, 700), p_hit=0.6, p_two=0.15,
                      p_n=0.02, xtra_mode="matesw"):
    """ksw_align2 tasks shaped like mem_matesw's (bwa/bwamem_pair.c:131-151):
    the mate (length from qlens) against a reference window of
    (high - low) + l_ms bases; with probability p_hit the window holds a
    diverged copy of the mate (a rescue), with p_two a second partial copy
    (the 2nd-best score path), otherwise random sequence.

    xtra_mode "matesw": XSUBO|XSTART|(l_ms*a < 250 ? XBYTE : 0)|min_seed_len*a
    (exactly what mem_matesw passes); "mix": also plain, XBYTE-saturating,
    XSTOP and XSTART-only calls.  Returns (tasks, qpool, tpool)."""
    tasks = np.zeros(n, abi.ALIGN2_TASK_DTYPE)
    qs, ts, qo, to = [], [], 0, 0
    for k in range(n):
        ql = int(qlens[int(rng.integers(0, len(qlens)))])
        q = rng.integers(0, 4, ql).astype(np.uint8)
        if p_n and ql:
            q[rng.random(ql) < p_n] = 4
        tl = int(rng.integers(win[0], win[1] + 1)) + ql
        t = rng.integers(0, 4, tl).astype(np.uint8)
        if rng.random() < p_hit and ql:
            m = _mutate(rng, q)
            if rng.random() < 0.25:  # partially outside the window: a clipped hit
                cut = int(rng.integers(0, max(1, len(m) // 2)))
                m = m[cut:] if rng.random() < 0.5 else m[:len(m) - cut]
            p = int(rng.integers(0, max(1, tl - len(m))))
            t[p:p + len(m)] = m[:tl - p]
            if rng.random() < p_two:
                m2 = _mutate(rng, q, sub=0.06)[: int(rng.integers(max(1, ql // 4), ql + 1))]
                p2 = int(rng.integers(0, max(1, tl - len(m2))))
                t[p2:p2 + len(m2)] = m2[:tl - p2]
        if p_n and tl:
            t[rng.random(tl) < p_n / 4] = 4
        xtra = abi.KSW_XSUBO | abi.KSW_XSTART | (abi.KSW_XBYTE if ql * a < 250 else 0) | (min_seed_len * a)
        if xtra_mode == "mix":
            u = rng.random()
            if u < 0.1:
                xtra = 0
            elif u < 0.2:
                xtra = abi.KSW_XBYTE | abi.KSW_XSTART
            elif u < 0.3:
                xtra = abi.KSW_XSTOP | int(rng.integers(1, 200)) | (abi.KSW_XBYTE if rng.random() < 0.5 else 0)
            elif u < 0.4:
                xtra = abi.KSW_XSUBO | abi.KSW_XSTART | int(rng.integers(0, 120))
            elif u < 0.5:
                xtra = abi.KSW_XSUBO | abi.KSW_XSTART | abi.KSW_XBYTE | int(rng.integers(0, 120))
        tasks[k] = (qo, to, ql, tl, xtra, 0)
        qs.append(q)
        ts.append(t)
        qo += ql
        to += tl
    cat = lambda v: np.concatenate(v).astype(np.uint8) if v else np.zeros(0, np.uint8)  # noqa: E731
    return tasks, cat(qs), cat(ts)
