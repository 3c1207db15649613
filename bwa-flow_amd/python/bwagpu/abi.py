"""ctypes mirror of include/bwagpu.h (the engine's C ABI) + numpy record dtypes.

The record dtypes are byte-for-byte the reference's structs:
  SEED_DTYPE   == mem_seed_t   (src/bwa_wrapper.h:62-66, 24 B)
  ALNREG_DTYPE == mem_alnreg_t (bwa/bwamem.h:60-79, 88 B)
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.normpath(os.path.join(HERE, "..", ".."))  # bwa-flow_amd/
REPO_ROOT = os.path.normpath(os.path.join(PKG_ROOT, ".."))
LIB_DIR = os.path.join(PKG_ROOT, "lib")

ABI_VERSION = 1
OK, E_INVAL, E_NOMEM, E_DEVICE, E_HANG, E_RESULTS, E_UNSUPPORTED, E_NODEVICE = range(8)
ERR_NAMES = {
    OK: "OK", E_INVAL: "E_INVAL", E_NOMEM: "E_NOMEM", E_DEVICE: "E_DEVICE", E_HANG: "E_HANG",
    E_RESULTS: "E_RESULTS", E_UNSUPPORTED: "E_UNSUPPORTED", E_NODEVICE: "E_NODEVICE",
}
MAX_READ_LEN = 1023
NUM_SLOTS = 4

SEED_DTYPE = np.dtype([("rbeg", "<i8"), ("qbeg", "<i4"), ("len", "<i4"), ("score", "<i4"),
                       ("pad", "<i4")])
ALNREG_DTYPE = np.dtype([
    ("rb", "<i8"), ("re", "<i8"), ("qb", "<i4"), ("qe", "<i4"), ("rid", "<i4"), ("score", "<i4"),
    ("truesc", "<i4"), ("sub", "<i4"), ("alt_sc", "<i4"), ("csub", "<i4"), ("sub_n", "<i4"),
    ("w", "<i4"), ("seedcov", "<i4"), ("secondary", "<i4"), ("secondary_all", "<i4"),
    ("seedlen0", "<i4"), ("n_comp_is_alt", "<u4"), ("frac_rep", "<f4"), ("hash", "<u8")])
EXT_TASK_DTYPE = np.dtype([("qoff", "<i8"), ("toff", "<i8"), ("qlen", "<i4"), ("tlen", "<i4"),
                           ("w", "<i4"), ("end_bonus", "<i4"), ("zdrop", "<i4"), ("h0", "<i4")])
EXT_RES_DTYPE = np.dtype([("score", "<i4"), ("qle", "<i4"), ("tle", "<i4"), ("gtle", "<i4"),
                          ("gscore", "<i4"), ("max_off", "<i4")])
ALIGN2_TASK_DTYPE = np.dtype([("qoff", "<i8"), ("toff", "<i8"), ("qlen", "<i4"), ("tlen", "<i4"),
                              ("xtra", "<i4"), ("pad", "<i4")])
KSWR_DTYPE = np.dtype([("score", "<i4"), ("te", "<i4"), ("qe", "<i4"), ("score2", "<i4"), ("te2", "<i4"),
                       ("tb", "<i4"), ("qb", "<i4")])
KSW_XBYTE, KSW_XSTOP, KSW_XSUBO, KSW_XSTART = 0x10000, 0x20000, 0x40000, 0x80000
REG2ALN_TASK_DTYPE = np.dtype([("rb", "<i8"), ("re", "<i8"), ("qoff", "<i8"), ("l_seq", "<i4"), ("qb", "<i4"),
                               ("qe", "<i4"), ("truesc", "<i4"), ("w", "<i4"), ("pad", "<i4")])
ALN_DTYPE = np.dtype([("pos", "<i8"), ("rid", "<i4"), ("is_rev", "<i4"), ("n_cigar", "<i4"), ("NM", "<i4"),
                      ("md_len", "<i4"), ("score", "<i4"), ("w", "<i4"), ("status", "<i4")])
ALN_OK, ALN_NO_CIGAR, ALN_OVERFLOW, ALN_UNMAPPED = 0, 1, 2, 3
assert REG2ALN_TASK_DTYPE.itemsize == 48 and ALN_DTYPE.itemsize == 40
assert SEED_DTYPE.itemsize == 24 and ALNREG_DTYPE.itemsize == 88
assert ALIGN2_TASK_DTYPE.itemsize == 32 and KSWR_DTYPE.itemsize == 28
assert EXT_TASK_DTYPE.itemsize == 40 and EXT_RES_DTYPE.itemsize == 24


class Opt(C.Structure):
    """bwagpu_opt_t: the mem_opt_t fields (bwa/bwamem.h:26-58) the path reads."""
    _fields_ = [("a", C.c_int32), ("b", C.c_int32), ("o_del", C.c_int32), ("e_del", C.c_int32),
                ("o_ins", C.c_int32), ("e_ins", C.c_int32), ("pen_clip5", C.c_int32),
                ("pen_clip3", C.c_int32), ("w", C.c_int32), ("zdrop", C.c_int32),
                ("mat", C.c_int8 * 25), ("pad_", C.c_int8 * 3)]


class Bns(C.Structure):
    _fields_ = [("l_pac", C.c_int64), ("n_seqs", C.c_int32), ("pad_", C.c_int32),
                ("ann_offset", C.c_void_p), ("ann_len", C.c_void_p)]


class BatchC(C.Structure):
    _fields_ = [("n_reads", C.c_int32), ("n_chains", C.c_int32), ("n_seeds", C.c_int32),
                ("pad_", C.c_int32), ("seq_bytes", C.c_int64), ("seq_off", C.c_void_p),
                ("seq", C.c_void_p), ("read_chain_off", C.c_void_p), ("chain_seed_off", C.c_void_p),
                ("chain_rid", C.c_void_p), ("chain_frac_rep", C.c_void_p), ("seeds", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double), ("total_ms", C.c_double), ("cells", C.c_int64),
                ("rows", C.c_int64), ("ext_calls", C.c_int64), ("h2d_bytes", C.c_int64),
                ("d2h_bytes", C.c_int64)]


class BwtC(C.Structure):
    """bwagpu_bwt_t == bwt_t's header + occurrence words (bwa/bwt.h:46-57)"""
    _fields_ = [("primary", C.c_uint64), ("L2", C.c_uint64 * 5), ("seq_len", C.c_uint64),
                ("bwt_size", C.c_uint64), ("bwt", C.c_void_p), ("sa_intv", C.c_int32), ("pad_", C.c_int32),
                ("n_sa", C.c_uint64), ("sa", C.c_void_p)]


class SeedOpt(C.Structure):
    """bwagpu_seedopt_t: mem_opt_t's seeding fields (bwamem.c:62-72)"""
    _fields_ = [("min_seed_len", C.c_int32), ("split_width", C.c_int32), ("max_mem_intv", C.c_int32),
                ("split_factor", C.c_float)]


INTV_DTYPE = np.dtype([("x", "<u8", (3,)), ("info", "<u8")])  # bwagpu_intv_t == bwtintv_t
assert INTV_DTYPE.itemsize == 32

# bwagpu_chain_t: mem_chain_t (bwa/bwamem.c:180-186) without its seed vector
CHAIN_DTYPE = np.dtype([("pos", "<i8"), ("rid", "<i4"), ("n", "<i4"), ("w", "<i4"), ("kept", "<i4"),
                        ("first", "<i4"), ("is_alt", "<i4"), ("frac_rep", "<f4"), ("pad_", "<i4")])
assert CHAIN_DTYPE.itemsize == 40


class ChainOpt(C.Structure):
    """bwagpu_chainopt_t: mem_opt_t's chaining fields (bwamem.c:62-72)"""
    _fields_ = [("max_occ", C.c_int32), ("max_chain_gap", C.c_int32), ("min_chain_weight", C.c_int32),
                ("max_chain_extend", C.c_int32), ("mask_level", C.c_float), ("drop_ratio", C.c_float)]


class ChainsC(C.Structure):
    """bwagpu_chains_t: a batch's chains in the bwagpu_batch_t layout"""
    _fields_ = [("n_reads", C.c_int32), ("n_chains", C.c_int32), ("n_seeds", C.c_int64),
                ("read_chain_off", C.c_void_p), ("chain_seed_off", C.c_void_p), ("chains", C.c_void_p),
                ("seeds", C.c_void_p)]


def default_chainopt() -> dict:
    """mem_opt_init's chaining defaults (bwa/bwamem.c:62-72)"""
    return dict(max_occ=500, max_chain_gap=10000, min_chain_weight=0, max_chain_extend=1 << 30, mask_level=0.5,
                drop_ratio=0.5)

# every entry point declared in include/bwagpu.h: name -> (restype, argtypes)
_VP = C.c_void_p
PROTOS = {
    "bwagpu_abi_version": (C.c_int, []),
    "bwagpu_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "bwagpu_create": (C.c_int, [C.c_int, C.POINTER(Opt), C.POINTER(Bns), _VP, C.POINTER(_VP)]),
    "bwagpu_create_resident": (C.c_int, [C.c_int, C.POINTER(Opt), C.POINTER(Bns), _VP, C.POINTER(_VP)]),
    "bwagpu_destroy": (C.c_int, [_VP]),
    "bwagpu_last_error": (C.c_char_p, [_VP]),
    "bwagpu_set_watchdog_ms": (C.c_int, [_VP, C.c_int]),
    "bwagpu_chain2aln_submit": (C.c_int, [_VP, C.c_int, C.POINTER(BatchC)]),
    "bwagpu_chain2aln_wait": (C.c_int, [_VP, C.c_int, _VP, _VP]),
    "bwagpu_chain2aln_stage": (C.c_int, [_VP, C.c_int, C.c_int32, C.c_int32, C.c_int32, C.c_int64,
                                         C.POINTER(BatchC)]),
    "bwagpu_chain2aln_results": (C.c_int, [_VP, C.c_int, C.POINTER(_VP), C.POINTER(_VP)]),
    "bwagpu_chain2aln_results_dense": (C.c_int, [_VP, C.c_int, C.POINTER(_VP), C.POINTER(_VP), C.POINTER(_VP)]),
    "bwagpu_chain2aln": (C.c_int, [_VP, C.POINTER(BatchC), _VP, _VP]),
    "bwagpu_chain2aln_device": (C.c_int, [_VP, C.POINTER(BatchC), _VP, _VP, _VP, _VP]),
    "bwagpu_extend_batch": (C.c_int, [_VP, C.c_int32, _VP, _VP, C.c_int64, _VP, C.c_int64, _VP]),
    "bwagpu_align2_batch": (C.c_int, [_VP, C.c_int32, _VP, _VP, C.c_int64, _VP, C.c_int64, _VP]),
    "bwagpu_align2_device": (C.c_int, [_VP, C.c_int32, _VP, _VP, _VP, _VP, _VP, _VP]),
    "bwagpu_reg2aln_batch": (C.c_int, [_VP, C.c_int32, _VP, _VP, C.c_int64, C.c_int32, C.c_int32, _VP, _VP, _VP]),
    "bwagpu_last_stats": (C.c_int, [_VP, C.c_int, C.POINTER(Stats)]),
    "bwagpu_debug_set_trace": (C.c_int, [_VP, _VP]),
    "bwagpu_prof_start": (C.c_int, [_VP, C.c_int]),
    "bwagpu_debug_fail_wait": (C.c_int, [_VP, C.c_int, C.c_int]),
    "bwagpu_debug_spec_counters": (C.c_int, [_VP, _VP, _VP]),
    "bwagpu_debug_occupancy": (C.c_int, [_VP, _VP, _VP]),
    "bwagpu_debug_spec_ext": (C.c_int, [_VP, _VP, _VP, C.c_int32]),
    "bwagpu_prof_read": (C.c_int, [_VP, C.POINTER(C.c_double), C.POINTER(C.c_int32)]),
    "bwagpu_prof_intervals": (C.c_int, [_VP, _VP, _VP, C.c_int32, C.POINTER(C.c_int32)]),
    "bwagpu_set_bwt": (C.c_int, [_VP, C.POINTER(BwtC)]),
    "bwagpu_debug_seed_budget": (C.c_int, [_VP, C.c_int32]),
    "bwagpu_debug_sup_shift": (C.c_int, [_VP, C.c_int32]),
    "bwagpu_set_device_read_len": (C.c_int, [_VP, C.c_int32]),
    "bwagpu_debug_ext_form": (C.c_int, [C.c_int]),
    "bwagpu_ctx_ext_form": (C.c_int, [_VP, C.c_int]),
    "bwagpu_ctx_row_bound": (C.c_int, [_VP, C.c_int]),
    "bwagpu_debug_ext_kernel": (C.c_int, [_VP, C.c_int32]),
    "bwagpu_streams_concurrent": (C.c_int, [_VP, _VP]),
    "bwagpu_bwt_sa": (C.c_int, [_VP, C.c_int64, _VP, _VP]),
    "bwagpu_sw_stream": (C.c_int, [_VP, _VP, C.c_int64, _VP, C.c_int32, C.POINTER(C.c_int32)]),
    "bwagpu_collect_intv": (C.c_int, [_VP, C.POINTER(SeedOpt), C.c_int32, _VP, _VP, C.c_int32, _VP, C.c_int64,
                                       _VP]),
    "bwagpu_set_alt": (C.c_int, [_VP, _VP]),
    "bwagpu_seqs2chains": (C.c_int, [_VP, C.POINTER(SeedOpt), C.POINTER(ChainOpt), C.c_int32, _VP, _VP, C.c_int32,
                                      C.POINTER(ChainsC)]),
    "bwagpu_seqs2regions": (C.c_int, [_VP, C.POINTER(SeedOpt), C.POINTER(ChainOpt), C.c_int32, _VP, _VP, _VP,
                                       C.POINTER(_VP), C.POINTER(C.c_int64)]),
}

_lib = None


def lib_path() -> str:
    return os.environ.get("BWAGPU_LIB", os.path.join(LIB_DIR, "libbwagpu.so"))


def load() -> C.CDLL:
    """Load the HIP engine.  Fails loudly: there is no CPU fallback."""
    global _lib
    if _lib is not None:
        return _lib
    p = lib_path()
    # one HIP runtime per process: when PyTorch is present its bundled
    # libamdhip64.so.7 must be the one our library binds to (same soname), so
    # import it first; a second runtime would hide the GPU from torch.
    if os.environ.get("BWAGPU_NO_TORCH") != "1":
        try:
            import torch  # noqa: F401
        except Exception:
            pass
    if not os.path.exists(p):
        raise RuntimeError(f"bwagpu: HIP engine library missing at {p}; run __graft_entry__.build()")
    lib = C.CDLL(p)
    for name, (res, args) in PROTOS.items():
        if name.startswith("bwagpu_debug_") and not hasattr(lib, name):
            continue  # an A/B build of an older tree (BWAGPU_LIB) may lack a newer diagnostic
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.bwagpu_abi_version() != ABI_VERSION:
        raise RuntimeError("bwagpu: ABI version mismatch")
    _lib = lib
    return lib


def opt_from_dict(d: dict) -> Opt:
    o = Opt()
    for k in ("a", "b", "o_del", "e_del", "o_ins", "e_ins", "pen_clip5", "pen_clip3", "w", "zdrop"):
        setattr(o, k, int(d[k]))
    mat = d.get("mat")
    if mat is None:
        mat = fill_scmat(int(d["a"]), int(d["b"]))
    for i in range(25):
        o.mat[i] = int(mat[i])
    return o


def fill_scmat(a: int, b: int) -> np.ndarray:
    """bwa_fill_scmat (bwa/bwa.c:109-118): a on the diagonal, -b off it, -1 for N."""
    m = np.full((5, 5), -1, np.int8)
    for i in range(4):
        for j in range(4):
            m[i, j] = a if i == j else -b
    return m.reshape(-1)


def default_opt() -> dict:
    """mem_opt_init defaults (bwa/bwamem.c:48-84)."""
    return dict(a=1, b=4, o_del=6, e_del=1, o_ins=6, e_ins=1, pen_clip5=5, pen_clip3=5, w=100,
                zdrop=100, mat=fill_scmat(1, 4))
