"""TEST INFRASTRUCTURE ONLY — ctypes access to the CPU checkers.

  liboracle.so         our clean-room C restatement (oracle/ksw_ext.c, chain2aln.c)
  _ref/libbwaref.so    the reference's own bwa C (compiled from /root/reference/bwa
                       by oracle/Makefile) behind ref_shim.c

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module.  The product (bwa-flow_amd/) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "bwa-flow_amd", "python"))
from bwagpu import abi  # noqa: E402  (record dtypes / ABI structs only)
from bwagpu.engine import Batch, _ptr  # noqa: E402

_VP = C.c_void_p
_libs: dict = {}


def _load(name: str, path: str):
    if name in _libs:
        return _libs[name]
    if not os.path.exists(path):
        return None
    lib = C.CDLL(path)
    _libs[name] = lib
    return lib


def oracle_lib():
    lib = _load("oracle", os.path.join(HERE, "liboracle.so"))
    if lib is None:
        raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle`")
    lib.oracle_chain2aln_batch.argtypes = [C.POINTER(abi.Opt), C.POINTER(abi.Bns), _VP, C.POINTER(abi.BatchC),
                                           _VP, _VP, C.c_int, _VP]
    lib.oracle_chain2aln_batch.restype = C.c_int
    lib.oracle_extend_batch.argtypes = [C.POINTER(abi.Opt), C.c_int32, _VP, _VP, _VP, _VP, _VP]
    lib.oracle_extend_batch.restype = C.c_int
    lib.oracle_extend_batch_bounded.argtypes = [C.POINTER(abi.Opt), C.c_int32, _VP, _VP, _VP, _VP, _VP]
    lib.oracle_extend_batch_bounded.restype = C.c_int
    lib.oracle_align2_batch.argtypes = [C.POINTER(abi.Opt), C.c_int32, _VP, _VP, _VP, _VP, _VP]
    lib.oracle_align2_batch.restype = C.c_int
    lib.oracle_reg2aln_batch.argtypes = [C.POINTER(abi.Opt), C.POINTER(abi.Bns), _VP, C.c_int32, _VP, _VP,
                                         C.c_int, C.c_int, _VP, _VP, _VP]
    lib.oracle_reg2aln_batch.restype = C.c_int
    lib.oracle_collect_intv.argtypes = [_VP, _VP, _VP, C.c_float, C.c_int, _VP, _VP, C.c_int]
    lib.oracle_collect_intv.restype = C.c_int
    lib.oracle_bwt_sa.argtypes = [_VP, _VP, _VP, C.c_int, C.c_uint64]
    lib.oracle_bwt_sa.restype = C.c_uint64
    lib.oracle_seqs2chains.argtypes = [C.POINTER(ChainEnv), C.c_int32, _VP, _VP, C.c_int, _VP, C.POINTER(ChainsOut)]
    lib.oracle_seqs2chains.restype = C.c_int
    lib.oracle_fpga_pack.argtypes = [C.POINTER(abi.Opt), C.POINTER(abi.Bns), C.POINTER(abi.BatchC), _VP, C.c_int64,
                                     C.c_int32, C.POINTER(C.c_int32), _VP, _VP]
    lib.oracle_fpga_pack.restype = C.c_int64
    lib.oracle_fpga_sw.argtypes = [C.POINTER(abi.Opt), C.POINTER(abi.Bns), _VP, _VP, C.c_int64, _VP, C.c_int32,
                                   C.POINTER(C.c_int32)]
    lib.oracle_fpga_sw.restype = C.c_int
    return lib


def ref_lib():
    """the reference's own code, or None when _ref/ was not built/shipped"""
    lib = _load("ref", os.path.join(HERE, "_ref", "libbwaref.so"))
    if lib is None:
        return None
    lib.ref_chain2aln_batch.argtypes = [C.POINTER(abi.Opt), C.POINTER(abi.Bns), _VP, C.POINTER(abi.BatchC),
                                        _VP, _VP, C.c_int]
    lib.ref_chain2aln_batch.restype = C.c_int
    lib.ref_extend_batch.argtypes = [C.POINTER(abi.Opt), C.c_int32, _VP, _VP, _VP, _VP]
    lib.ref_extend_batch.restype = C.c_int
    lib.ref_abi_check.restype = C.c_int
    if hasattr(lib, "ref_reg2aln_batch"):
        lib.ref_reg2aln_batch.argtypes = [C.POINTER(abi.Opt), C.POINTER(abi.Bns), _VP, C.c_int32, _VP, _VP,
                                          C.c_int, C.c_int, _VP, _VP, _VP]
        lib.ref_reg2aln_batch.restype = C.c_int
    if hasattr(lib, "ref_align2_batch"):
        lib.ref_align2_batch.argtypes = [C.POINTER(abi.Opt), C.c_int32, _VP, _VP, _VP, _VP]
        lib.ref_align2_batch.restype = C.c_int
    return lib


class Ref:
    """reference genome in bwa's form: forward 2-bit pac + contig table"""

    def __init__(self, l_pac, ann_offset, ann_len, pac):
        self.l_pac = int(l_pac)
        self.ann_offset = np.ascontiguousarray(ann_offset, np.int64)
        self.ann_len = np.ascontiguousarray(ann_len, np.int32)
        self.pac = np.ascontiguousarray(pac, np.uint8)
        self.bns = abi.Bns(self.l_pac, len(self.ann_offset), 0, _ptr(self.ann_offset), _ptr(self.ann_len))


def chain2aln(which: str, opt: dict, ref: Ref, batch: Batch, n_threads: int = 1):
    """CPU mem_chain2aln over a batch -> (regs, n, stats[cells, rows, calls] or None)"""
    o = abi.opt_from_dict(opt)
    regs = np.zeros(max(batch.n_seeds, 1), abi.ALNREG_DTYPE)
    n = np.zeros(max(batch.n_reads, 1), np.int32)
    bc = batch.to_c()
    if which == "oracle":
        st = np.zeros(3, np.int64)
        rc = oracle_lib().oracle_chain2aln_batch(C.byref(o), C.byref(ref.bns), _ptr(ref.pac), C.byref(bc),
                                                 _ptr(regs), _ptr(n), n_threads, _ptr(st))
    elif which == "ref":
        lib = ref_lib()
        if lib is None:
            raise RuntimeError("oracle/_ref/libbwaref.so not available")
        st = None
        rc = lib.ref_chain2aln_batch(C.byref(o), C.byref(ref.bns), _ptr(ref.pac), C.byref(bc), _ptr(regs),
                                     _ptr(n), n_threads)
    else:
        raise ValueError(which)
    if rc != 0:
        raise RuntimeError(f"{which} chain2aln failed rc={rc}")
    return regs[:batch.n_seeds], n[:batch.n_reads], st


def ref_seqs2chains(prefix: str, seq_off, seq, n_threads: int = 1):
    """the REFERENCE's SeqsToChains (mem_chain -> mem_chain_flt ->
    mem_flt_chained_seeds, src/bwa_wrapper.cpp:105-115) over a batch of reads
    against the bwa index at `prefix` (oracle/_ref/libbwaref.so
    ref_seqs2chains_batch) -> (read_chain_off, chain_rid, chain_frac_rep,
    chain_seed_off, seeds) in the bwagpu_batch_t layout"""
    lib = ref_lib()
    if lib is None:
        raise RuntimeError("oracle/_ref/libbwaref.so not available")
    fn = lib.ref_seqs2chains_batch
    fn.restype = C.c_int
    fn.argtypes = [C.c_char_p, C.c_int32, _VP, _VP, C.c_int, _VP, C.c_int64, _VP, _VP, _VP, C.c_int64, _VP,
                   C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    seq_off = np.ascontiguousarray(seq_off, np.int64)
    seq = np.ascontiguousarray(seq, np.uint8)
    n = len(seq_off) - 1
    cap_c, cap_s = 4 * n + 16, 16 * n + 64
    while True:
        rco = np.zeros(n + 1, np.int32)
        rid = np.zeros(cap_c, np.int32)
        fr = np.zeros(cap_c, np.float32)
        cso = np.zeros(cap_c + 1, np.int32)
        sd = np.zeros(cap_s, abi.SEED_DTYPE)
        nc, ns = C.c_int64(), C.c_int64()
        rc = fn(prefix.encode(), n, _ptr(seq_off), _ptr(seq), int(n_threads), _ptr(rco), cap_c, _ptr(rid), _ptr(fr),
                _ptr(cso), cap_s, _ptr(sd), C.byref(nc), C.byref(ns))
        if rc == -2:
            cap_c, cap_s = int(nc.value) + 16, int(ns.value) + 64
            continue
        if rc != 0:
            raise RuntimeError(f"ref_seqs2chains_batch rc={rc} (index {prefix})")
        c, k = int(nc.value), int(ns.value)
        return rco, rid[:c], fr[:c], cso[:c + 1], sd[:k]


def extend(which: str, opt: dict, tasks, qpool, tpool):
    o = abi.opt_from_dict(opt)
    tasks = np.ascontiguousarray(tasks, abi.EXT_TASK_DTYPE)
    qpool = np.ascontiguousarray(qpool, np.uint8)
    tpool = np.ascontiguousarray(tpool, np.uint8)
    res = np.zeros(max(len(tasks), 1), abi.EXT_RES_DTYPE)
    if which in ("oracle", "oracle_bounded"):  # oracle_bounded: with the GPU kernels' row bound (tests)
        cells = np.zeros(2, np.int64)
        fn = oracle_lib().oracle_extend_batch if which == "oracle" else oracle_lib().oracle_extend_batch_bounded
        fn(C.byref(o), len(tasks), _ptr(tasks), _ptr(qpool), _ptr(tpool), _ptr(res), _ptr(cells))
        return res[:len(tasks)], cells
    lib = ref_lib()
    if lib is None:
        raise RuntimeError("oracle/_ref/libbwaref.so not available")
    lib.ref_extend_batch(C.byref(o), len(tasks), _ptr(tasks), _ptr(qpool), _ptr(tpool), _ptr(res))
    return res[:len(tasks)], None


def align2(which: str, opt: dict, tasks, qpool, tpool):
    """ksw_align2 over a task batch -> (kswr records, cells[cells, rows] or None)"""
    o = abi.opt_from_dict(opt)
    tasks = np.ascontiguousarray(tasks, abi.ALIGN2_TASK_DTYPE)
    qpool = np.ascontiguousarray(qpool, np.uint8)
    tpool = np.ascontiguousarray(tpool, np.uint8)
    res = np.zeros(max(len(tasks), 1), abi.KSWR_DTYPE)
    if which == "oracle":
        cells = np.zeros(2, np.int64)
        oracle_lib().oracle_align2_batch(C.byref(o), len(tasks), _ptr(tasks), _ptr(qpool), _ptr(tpool),
                                         _ptr(res), _ptr(cells))
        return res[:len(tasks)], cells
    lib = ref_lib()
    if lib is None or not hasattr(lib, "ref_align2_batch"):
        raise RuntimeError("oracle/_ref/libbwaref.so (with ref_align2_batch) not available")
    lib.ref_align2_batch(C.byref(o), len(tasks), _ptr(tasks), _ptr(qpool), _ptr(tpool), _ptr(res))
    return res[:len(tasks)], None


def reg2aln(which: str, opt: dict, ref: Ref, tasks, qpool, max_ops: int = 64, max_md: int = 512):
    """mem_reg2aln's CIGAR part per job -> (aln records, cigar [n, max_ops] u32, md [n, max_md] bytes)"""
    o = abi.opt_from_dict(opt)
    tasks = np.ascontiguousarray(tasks, abi.REG2ALN_TASK_DTYPE)
    qpool = np.ascontiguousarray(qpool, np.uint8)
    n = len(tasks)
    out = np.zeros(max(n, 1), abi.ALN_DTYPE)
    cig = np.zeros((max(n, 1), max_ops), np.uint32)
    md = np.zeros((max(n, 1), max_md), np.uint8)
    if which == "oracle":
        f = oracle_lib().oracle_reg2aln_batch
    else:
        lib = ref_lib()
        if lib is None or not hasattr(lib, "ref_reg2aln_batch"):
            raise RuntimeError("oracle/_ref/libbwaref.so (with ref_reg2aln_batch) not available")
        f = lib.ref_reg2aln_batch
    f(C.byref(o), C.byref(ref.bns), _ptr(ref.pac), n, _ptr(tasks), _ptr(qpool), max_ops, max_md, _ptr(out),
      _ptr(cig), _ptr(md))
    return out[:n], cig[:n], md[:n]


def collect_intv(bwt_hdr, bwt_words, opt_i32, split_factor, seq_off, seq, cap: int = 512):
    """mem_collect_intv per read with the restatement (oracle/seed.c) ->
    (counts int32[n], intervals uint64[sum, 4] in the reference's order)"""
    hdr = np.ascontiguousarray(np.asarray(bwt_hdr, np.int64)[:7])
    words = np.ascontiguousarray(bwt_words, np.uint32)
    ov = np.ascontiguousarray(opt_i32, np.int32)
    seq = np.ascontiguousarray(seq, np.uint8)
    lib = oracle_lib()
    buf = np.zeros((cap, 4), np.uint64)
    counts, out = [], []
    for r in range(len(seq_off) - 1):
        q = seq[seq_off[r]:seq_off[r + 1]]
        q = np.ascontiguousarray(q)
        n = lib.oracle_collect_intv(_ptr(hdr), _ptr(words), _ptr(ov), float(split_factor), len(q), _ptr(q),
                                    _ptr(buf), len(buf))
        if n > len(buf):  # a repetitive read: again with room for all of them
            buf = np.zeros((n, 4), np.uint64)
            n = lib.oracle_collect_intv(_ptr(hdr), _ptr(words), _ptr(ov), float(split_factor), len(q), _ptr(q),
                                        _ptr(buf), len(buf))
        counts.append(n)
        out.append(buf[:n].copy())
    return np.array(counts, np.int32), (np.concatenate(out) if out else np.zeros((0, 4), np.uint64))


def bwt_sa(bwt_hdr, bwt_words, sa, sa_intv, ks):
    """bwt_sa per BWT position with the restatement (oracle/seed.c)"""
    hdr = np.ascontiguousarray(np.asarray(bwt_hdr, np.int64)[:7])
    words = np.ascontiguousarray(bwt_words, np.uint32)
    sa = np.ascontiguousarray(sa, np.uint64)
    lib = oracle_lib()
    return np.array([lib.oracle_bwt_sa(_ptr(hdr), _ptr(words), _ptr(sa), int(sa_intv), int(k)) for k in ks], np.uint64)


class ChainOptO(C.Structure):  # oracle_chainopt_t
    _fields_ = [("max_occ", C.c_int32), ("max_chain_gap", C.c_int32), ("min_chain_weight", C.c_int32),
                ("max_chain_extend", C.c_int32), ("mask_level", C.c_float), ("drop_ratio", C.c_float),
                ("min_seed_len", C.c_int32)]


class ChainEnv(C.Structure):  # oracle_chain_env_t
    _fields_ = [("opt", C.POINTER(abi.Opt)), ("copt", C.POINTER(ChainOptO)), ("bns", C.POINTER(abi.Bns)),
                ("pac", _VP), ("is_alt", _VP), ("bwt_hdr", _VP), ("bwt_words", _VP), ("sa", _VP),
                ("sa_intv", C.c_int32), ("seedopt", _VP), ("split_factor", C.c_float)]


class ChainsOut(C.Structure):  # oracle_chains_t
    _fields_ = [("chains", _VP), ("seeds", _VP), ("cap_chains", C.c_int64), ("cap_seeds", C.c_int64),
                ("n_chains", C.c_int64), ("n_seeds", C.c_int64)]


def seqs2chains(opt: dict, copt: dict, seedopt, split_factor, ref: Ref, is_alt, bwt_hdr, bwt_words, sa, sa_intv,
                seq_off, seq, raw: bool = False):
    """SeqsToChains' chaining per read with the restatement (oracle/chain.c) ->
    (read_chain_off int32[n+1], chains CHAIN_DTYPE, chain_seed_off int32, seeds SEED_DTYPE)"""
    o = abi.opt_from_dict(opt)
    co = ChainOptO(int(copt["max_occ"]), int(copt["max_chain_gap"]), int(copt["min_chain_weight"]),
                   int(copt["max_chain_extend"]), float(copt["mask_level"]), float(copt["drop_ratio"]),
                   int(seedopt[0]))
    keep = dict(hdr=np.ascontiguousarray(np.asarray(bwt_hdr, np.int64)[:7]),
                words=np.ascontiguousarray(bwt_words, np.uint32), sa=np.ascontiguousarray(sa, np.uint64),
                so=np.ascontiguousarray(seedopt, np.int32)[:3].copy(),
                alt=None if is_alt is None else np.ascontiguousarray(is_alt, np.uint8),
                seq_off=np.ascontiguousarray(seq_off, np.int64), seq=np.ascontiguousarray(seq, np.uint8))
    env = ChainEnv(C.pointer(o), C.pointer(co), C.pointer(ref.bns), _ptr(ref.pac),
                   None if keep["alt"] is None else _ptr(keep["alt"]), _ptr(keep["hdr"]), _ptr(keep["words"]),
                   _ptr(keep["sa"]), int(sa_intv), _ptr(keep["so"]), float(split_factor))
    n = len(keep["seq_off"]) - 1
    rco = np.zeros(n + 1, np.int32)
    cap_c, cap_s = 4 * n + 16, 16 * n + 64
    while True:
        ch = np.zeros(cap_c, abi.CHAIN_DTYPE)
        sd = np.zeros(cap_s, abi.SEED_DTYPE)
        out = ChainsOut(_ptr(ch), _ptr(sd), cap_c, cap_s, 0, 0)
        rc = oracle_lib().oracle_seqs2chains(C.byref(env), n, _ptr(keep["seq_off"]), _ptr(keep["seq"]), int(raw),
                                             _ptr(rco), C.byref(out))
        if rc == 0:
            break
        cap_c, cap_s = int(out.n_chains), int(out.n_seeds)
    ch = ch[:out.n_chains]
    cso = np.concatenate([[0], np.cumsum(ch["n"])]).astype(np.int32)
    return rco, ch, cso, sd[:out.n_seeds]


def fpga_pack(opt: dict, ref: Ref, batch: Batch):
    """packReadData over a batch (FPGAPipeline.cpp:194-343) -> (words int32, n_tasks, packed[n_reads],
    task_seed[n_tasks]: the batch seed index of each task)"""
    o = abi.opt_from_dict(opt)
    bc = batch.to_c()
    cap_w = 16 + 4 * batch.n_reads + int(batch.seq_off[-1]) // 8 + 5 * batch.n_chains + 5 * batch.n_seeds
    words = np.zeros(max(cap_w, 1), np.int32)
    packed = np.zeros(max(batch.n_reads, 1), np.int32)
    task_seed = np.zeros(max(batch.n_seeds, 1), np.int32)
    nt = C.c_int32(0)
    nw = oracle_lib().oracle_fpga_pack(C.byref(o), C.byref(ref.bns), C.byref(bc), _ptr(words), cap_w,
                                       max(batch.n_seeds, 1), C.byref(nt), _ptr(packed), _ptr(task_seed))
    if nw < 0:
        raise RuntimeError("fpga_pack: buffer too small")
    return words[:nw], nt.value, packed[:batch.n_reads], task_seed[:nt.value]


def fpga_sw(opt: dict, ref: Ref, words, cap_tasks: int):
    """the records bwagpu_sw_stream must return -> int16[n, 10], or None for a malformed stream"""
    o = abi.opt_from_dict(opt)
    words = np.ascontiguousarray(words, np.int32)
    out = np.zeros((max(cap_tasks, 1), 10), np.int16)
    nt = C.c_int32(0)
    rc = oracle_lib().oracle_fpga_sw(C.byref(o), C.byref(ref.bns), _ptr(ref.pac), _ptr(words), len(words),
                                     _ptr(out), int(cap_tasks), C.byref(nt))
    return None if rc != 0 else out[:nt.value]
