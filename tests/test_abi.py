"""CPU: the C-ABI library builds for gfx950, loads, and exports exactly what
include/bwagpu.h and include/bwagpu_debug.h declare; the Python/numpy mirrors match the C layouts.
No compute calls here (no GPU in the CPU tier)."""
import ctypes as C
import os
import re
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

from bwagpu import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "include", "bwagpu.h")
# the tuning / test / profiling entries live in a header of their own
DBG_HDR = os.path.join(REPO, "include", "bwagpu_debug.h")


def declared_functions():
    txt = open(HDR).read() + open(DBG_HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(bwagpu_\w+)\s*\(", txt, re.M)))


def test_header_declares_entry_points():
    fns = declared_functions()
    assert set(fns) == set(abi.PROTOS), f"header vs ctypes table: {set(fns) ^ set(abi.PROTOS)}"


def test_library_exports_every_declared_symbol():
    lib = abi.load()
    for fn in declared_functions():
        assert hasattr(lib, fn), fn
    out = subprocess.run(["nm", "-D", "--defined-only", abi.lib_path()], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (bwagpu_\w+)", out))
    assert exported == set(declared_functions())


def test_library_is_gfx950_code_object():
    # llvm-objdump extracts the bundled code objects next to its input: work on a copy
    with tempfile.TemporaryDirectory() as td:
        lib = os.path.join(td, "libbwagpu.so")
        shutil.copy(abi.lib_path(), lib)
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib],
                             capture_output=True, text=True, cwd=td)
    assert "gfx950" in (out.stdout + out.stderr)


def test_abi_version_and_no_device_on_cpu():
    lib = abi.load()
    assert lib.bwagpu_abi_version() == abi.ABI_VERSION
    n = C.c_int(-1)
    rc = lib.bwagpu_device_count(C.byref(n))
    if n.value == 0:
        assert rc == abi.E_NODEVICE
        ctx = C.c_void_p()
        o = abi.opt_from_dict(abi.default_opt())
        off = np.zeros(1, np.int64)
        ln = np.ones(1, np.int32) * 8
        bns = abi.Bns(8, 1, 0, off.ctypes.data, ln.ctypes.data)
        pac = np.zeros(3, np.uint8)
        assert lib.bwagpu_create(0, C.byref(o), C.byref(bns), pac.ctypes.data, C.byref(ctx)) == abi.E_NODEVICE


def test_null_arguments_are_rejected():
    lib = abi.load()
    assert lib.bwagpu_device_count(None) == abi.E_INVAL
    assert lib.bwagpu_destroy(None) == abi.E_INVAL
    assert lib.bwagpu_set_watchdog_ms(None, 5) == abi.E_INVAL
    assert lib.bwagpu_chain2aln(None, None, None, None) == abi.E_INVAL
    assert lib.bwagpu_last_error(None) == b"NULL context"
    assert lib.bwagpu_set_device_read_len(None, 150) == abi.E_INVAL


LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "bwagpu.h"
#define P(T, f) printf("%s %s %zu %zu\n", #T, #f, offsetof(T, f), sizeof(((T*)0)->f));
int main(void) {
  printf("sizes %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(bwagpu_opt_t), sizeof(bwagpu_seed_t),
         sizeof(bwagpu_alnreg_t), sizeof(bwagpu_bns_t), sizeof(bwagpu_batch_t), sizeof(bwagpu_ext_task_t),
         sizeof(bwagpu_ext_result_t), sizeof(bwagpu_stats_t));
  P(bwagpu_seed_t, rbeg) P(bwagpu_seed_t, qbeg) P(bwagpu_seed_t, len) P(bwagpu_seed_t, score)
  P(bwagpu_alnreg_t, rb) P(bwagpu_alnreg_t, re) P(bwagpu_alnreg_t, qb) P(bwagpu_alnreg_t, qe)
  P(bwagpu_alnreg_t, rid) P(bwagpu_alnreg_t, score) P(bwagpu_alnreg_t, truesc) P(bwagpu_alnreg_t, sub)
  P(bwagpu_alnreg_t, w) P(bwagpu_alnreg_t, seedcov) P(bwagpu_alnreg_t, seedlen0)
  P(bwagpu_alnreg_t, n_comp_is_alt) P(bwagpu_alnreg_t, frac_rep) P(bwagpu_alnreg_t, hash)
  P(bwagpu_ext_task_t, qoff) P(bwagpu_ext_task_t, toff) P(bwagpu_ext_task_t, qlen) P(bwagpu_ext_task_t, h0)
  P(bwagpu_ext_result_t, score) P(bwagpu_ext_result_t, max_off)
  return 0;
}
"""


def test_struct_layouts_match_numpy_and_ctypes():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "l.c")
        open(src, "w").write(LAYOUT_C)
        exe = os.path.join(d, "l")
        subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), src, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    sizes = list(map(int, out[0].split()[1:]))
    assert sizes == [C.sizeof(abi.Opt), 24, 88, C.sizeof(abi.Bns), C.sizeof(abi.BatchC), 40, 24, C.sizeof(abi.Stats)]
    dts = {"bwagpu_seed_t": abi.SEED_DTYPE, "bwagpu_alnreg_t": abi.ALNREG_DTYPE,
           "bwagpu_ext_task_t": abi.EXT_TASK_DTYPE, "bwagpu_ext_result_t": abi.EXT_RES_DTYPE}
    for line in out[1:]:
        if not line:
            continue
        t, f, off, sz = line.split()
        fo = dts[t].fields[f]
        assert fo[1] == int(off) and fo[0].itemsize == int(sz), (t, f)


def test_reference_struct_offsets():
    """mem_alnreg_t offsets measured on the reference build"""
    want = dict(rb=0, re=8, qb=16, qe=20, rid=24, score=28, truesc=32, sub=36, w=52, seedcov=56, seedlen0=68,
                frac_rep=76, hash=80)
    for k, v in want.items():
        assert abi.ALNREG_DTYPE.fields[k][1] == v


SAM_HDR = os.path.join(REPO, "include", "bwagpu_sam.h")
SAM_LIB = os.path.join(REPO, "bwa-flow_amd", "lib", "libgpusam.so")


def test_sam_cache_library_exports_its_header():
    """lib/libgpusam.so (the SAM-stage call cache) exports exactly what
    include/bwagpu_sam.h declares"""
    txt = open(SAM_HDR).read()
    declared = set(re.findall(r"^\s*(?:int|int64_t)\s*(bwagpu_samcache_\w+)\s*\(", txt, re.M))
    assert len(declared) == 7
    out = subprocess.run(["nm", "-D", "--defined-only", SAM_LIB], capture_output=True, text=True).stdout
    assert set(re.findall(r"\bT (bwagpu_\w+)", out)) == declared


def test_sam_cache_queues_misses_without_a_device():
    """host logic only (no flush): a miss answers with the placeholders the
    hooks rely on, a repeated call is not queued twice, bad arguments are
    negative codes distinct from hit (0) / miss (1)"""
    lib = C.CDLL(SAM_LIB)
    lib.bwagpu_samcache_create.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]
    lib.bwagpu_samcache_align2.argtypes = [C.c_void_p, C.c_int32, C.c_char_p, C.c_int32, C.c_char_p, C.c_int32,
                                           C.c_void_p]
    lib.bwagpu_samcache_reg2aln.argtypes = [C.c_void_p, C.c_int32, C.c_char_p, C.c_int64, C.c_int64, C.c_int32,
                                            C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.POINTER(C.c_void_p)]
    lib.bwagpu_samcache_stats.argtypes = [C.c_void_p, C.c_void_p]
    lib.bwagpu_samcache_clear.argtypes = [C.c_void_p]
    lib.bwagpu_samcache_destroy.argtypes = [C.c_void_p]
    c = C.c_void_p()
    # the cache keeps the context for flushes only; none happens here
    assert lib.bwagpu_samcache_create(C.c_void_p(1), 64, 512, C.byref(c)) == 0
    r = (C.c_int32 * 7)()
    q, t = bytes([0, 1, 2, 3] * 10), bytes([3, 2, 1, 0] * 50)
    for _ in range(2):
        assert lib.bwagpu_samcache_align2(c, len(q), q, len(t), t, 0x40000 | 30, r) == 1
        assert list(r) == [0, -1, -1, -1, -1, -1, -1]
    assert lib.bwagpu_samcache_align2(c, -1, q, len(t), t, 0, r) < 0
    aln = (C.c_int32 * 12)()
    cig = C.c_void_p()
    assert lib.bwagpu_samcache_reg2aln(c, len(q), q, 100, 140, 0, 40, 40, 5, aln, C.byref(cig)) == 1
    assert aln[9] == -1 and cig.value  # status, empty malloc'd block
    C.CDLL(None).free(cig)
    assert lib.bwagpu_samcache_reg2aln(c, len(q), q, -1, 140, 0, 40, 40, 5, aln, C.byref(cig)) < 0
    st = (C.c_int64 * 8)()
    assert lib.bwagpu_samcache_stats(c, st) == 0
    assert list(st) == [0, 2, 0, 1, 0, 0, 0, 0]
    assert lib.bwagpu_samcache_clear(c) == 0 and lib.bwagpu_samcache_destroy(c) == 0
