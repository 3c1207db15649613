"""Python host mirror of the engine: flattened read batches and a per-device
Engine wrapping the C ABI.  Used by tests, smoke() and bench.py; the C++ host
(bwa-flow_amd/host/) uses the same ABI directly."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import abi


class BwaGpuError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{abi.ERR_NAMES.get(code, code)}: {msg}")
        self.code = code


def _ptr(a: np.ndarray | None):
    return None if a is None or a.size == 0 else a.ctypes.data_as(C.c_void_p)


@dataclass
class Batch:
    """One ChainsRecord (src/Pipeline.h:46-57) in flattened form, see bwagpu_batch_t."""
    seq_off: np.ndarray         # int64 [n_reads+1]
    seq: np.ndarray             # uint8 nt4
    read_chain_off: np.ndarray  # int32 [n_reads+1]
    chain_seed_off: np.ndarray  # int32 [n_chains+1]
    chain_rid: np.ndarray       # int32 [n_chains]
    chain_frac_rep: np.ndarray  # float32 [n_chains]
    seeds: np.ndarray           # SEED_DTYPE [n_seeds]

    def __post_init__(self):
        self.seq_off = np.ascontiguousarray(self.seq_off, np.int64)
        self.seq = np.ascontiguousarray(self.seq, np.uint8)
        self.read_chain_off = np.ascontiguousarray(self.read_chain_off, np.int32)
        self.chain_seed_off = np.ascontiguousarray(self.chain_seed_off, np.int32)
        self.chain_rid = np.ascontiguousarray(self.chain_rid, np.int32)
        self.chain_frac_rep = np.ascontiguousarray(self.chain_frac_rep, np.float32)
        self.seeds = np.ascontiguousarray(self.seeds, abi.SEED_DTYPE)

    @property
    def n_reads(self) -> int:
        return len(self.seq_off) - 1

    @property
    def n_chains(self) -> int:
        return len(self.chain_seed_off) - 1

    @property
    def n_seeds(self) -> int:
        return len(self.seeds)

    def read_seed_off(self) -> np.ndarray:
        """first output slot of every read: chain_seed_off[read_chain_off[r]]"""
        return self.chain_seed_off[self.read_chain_off[:-1]]

    def to_c(self) -> abi.BatchC:
        b = abi.BatchC()
        b.n_reads, b.n_chains, b.n_seeds = self.n_reads, self.n_chains, self.n_seeds
        b.seq_bytes = int(self.seq_off[-1]) if self.n_reads >= 0 else 0
        b.seq_off = _ptr(self.seq_off)
        b.seq = _ptr(self.seq)
        b.read_chain_off = _ptr(self.read_chain_off)
        b.chain_seed_off = _ptr(self.chain_seed_off)
        b.chain_rid = _ptr(self.chain_rid)
        b.chain_frac_rep = _ptr(self.chain_frac_rep)
        b.seeds = _ptr(self.seeds)
        return b

    def subset(self, reads) -> "Batch":
        """a new batch holding the given reads (in the given order)"""
        reads = np.asarray(reads, np.int64)
        so, rco, cso = self.seq_off, self.read_chain_off, self.chain_seed_off
        seq_parts, seed_parts, rid, fr = [], [], [], []
        seq_off, rc_off, cs_off = [0], [0], [0]
        for r in reads:
            seq_parts.append(self.seq[so[r]:so[r + 1]])
            seq_off.append(seq_off[-1] + int(so[r + 1] - so[r]))
            for c in range(rco[r], rco[r + 1]):
                seed_parts.append(self.seeds[cso[c]:cso[c + 1]])
                cs_off.append(cs_off[-1] + int(cso[c + 1] - cso[c]))
                rid.append(self.chain_rid[c])
                fr.append(self.chain_frac_rep[c])
            rc_off.append(len(rid))
        return Batch(np.array(seq_off), np.concatenate(seq_parts) if seq_parts else np.zeros(0, np.uint8),
                     np.array(rc_off), np.array(cs_off), np.array(rid, np.int32), np.array(fr, np.float32),
                     np.concatenate(seed_parts) if seed_parts else np.zeros(0, abi.SEED_DTYPE))


def unflatten(batch: Batch, regs: np.ndarray, n: np.ndarray) -> list[np.ndarray]:
    """per-read region arrays (each the read's mem_alnreg_v contents in order)"""
    off = batch.read_seed_off()
    return [regs[off[r]:off[r] + n[r]] for r in range(batch.n_reads)]


def compact(batch: Batch, regs: np.ndarray, n: np.ndarray) -> np.ndarray:
    """concatenate the regions of all reads in read order"""
    n = np.asarray(n, np.int64)
    tot = int(n.sum())
    if tot == 0:
        return np.zeros(0, regs.dtype if regs is not None else abi.ALNREG_DTYPE)
    start = np.repeat(batch.read_seed_off().astype(np.int64), n)
    first = np.repeat(np.cumsum(n) - n, n)
    return regs[start + np.arange(tot, dtype=np.int64) - first]


class Engine:
    """One device context (bwagpu_create).  There is no CPU path behind it."""

    def __init__(self, device: int, opt: dict, l_pac: int, ann_offset, ann_len, pac=None,
                 pac_device_ptr: int | None = None):
        self.lib = abi.load()
        self.device = device
        self._args = (device, opt, l_pac, ann_offset, ann_len, pac, pac_device_ptr)
        self.opt = abi.opt_from_dict(opt)
        self._ann_off = np.ascontiguousarray(ann_offset, np.int64)
        self._ann_len = np.ascontiguousarray(ann_len, np.int32)
        self.bns = abi.Bns(int(l_pac), len(self._ann_off), 0, _ptr(self._ann_off), _ptr(self._ann_len))
        self.ctx = C.c_void_p()
        if pac_device_ptr is not None:
            rc = self.lib.bwagpu_create_resident(device, C.byref(self.opt), C.byref(self.bns),
                                                 C.c_void_p(pac_device_ptr), C.byref(self.ctx))
        else:
            self._pac = np.ascontiguousarray(pac, np.uint8)
            if len(self._pac) < int(l_pac) // 4 + 1:
                raise ValueError("pac shorter than l_pac/4+1 bytes")
            rc = self.lib.bwagpu_create(device, C.byref(self.opt), C.byref(self.bns), _ptr(self._pac),
                                        C.byref(self.ctx))
        if rc != abi.OK:
            raise BwaGpuError(rc, "bwagpu_create failed")

    def clone(self) -> "Engine":
        """another context on the same device with the same options and reference
        (a second stage worker); the FM-index is not carried over (set_bwt)"""
        return Engine(*self._args[:5], pac=self._args[5], pac_device_ptr=self._args[6])

    def close(self):
        if self.ctx:
            self.lib.bwagpu_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc != abi.OK:
            raise BwaGpuError(rc, f"{what}: {self.lib.bwagpu_last_error(self.ctx).decode()}")

    def set_watchdog_ms(self, ms: int):
        self._check(self.lib.bwagpu_set_watchdog_ms(self.ctx, int(ms)), "set_watchdog_ms")

    def chain2aln(self, batch: Batch):
        """-> (regs[n_seeds] ALNREG_DTYPE, n[n_reads] int32)"""
        regs = np.zeros(max(batch.n_seeds, 1), abi.ALNREG_DTYPE)
        n = np.zeros(max(batch.n_reads, 1), np.int32)
        bc = batch.to_c()
        self._check(self.lib.bwagpu_chain2aln(self.ctx, C.byref(bc), _ptr(regs), _ptr(n)), "chain2aln")
        return regs[:batch.n_seeds], n[:batch.n_reads]

    def submit(self, slot: int, batch: Batch):
        bc = batch.to_c()
        self._check(self.lib.bwagpu_chain2aln_submit(self.ctx, slot, C.byref(bc)), "submit")

    def wait(self, slot: int, batch: Batch, out=None):
        """-> (regs, n) as chain2aln; `out` = (regs, n) arrays of at least
        max(n_seeds, 1) / max(n_reads, 1) entries to reuse instead of fresh ones"""
        if out is None:
            regs = np.zeros(max(batch.n_seeds, 1), abi.ALNREG_DTYPE)
            n = np.zeros(max(batch.n_reads, 1), np.int32)
        else:
            regs, n = out
            if (regs.dtype != abi.ALNREG_DTYPE or n.dtype != np.int32 or not regs.flags.c_contiguous
                    or not n.flags.c_contiguous or len(regs) < max(batch.n_seeds, 1) or len(n) < max(batch.n_reads, 1)):
                raise ValueError("wait: out arrays too small or of the wrong dtype/layout")
        self._check(self.lib.bwagpu_chain2aln_wait(self.ctx, slot, _ptr(regs), _ptr(n)), "wait")
        return regs[:batch.n_seeds], n[:batch.n_reads]

    def wait_dense(self, slot: int, batch: Batch, out=None):
        """-> (regs, n): the slot's results in read order without slot gaps
        (bwagpu_chain2aln_results_dense: only these regions crossed PCIe).
        out=None: numpy views onto the slot's pinned result buffers, valid
        until the slot's next submit (no host copy); `out` = (regs, n) arrays
        to copy into instead"""
        self._check(self.lib.bwagpu_chain2aln_wait(self.ctx, slot, None, None), "wait")
        rp, np_, op = C.c_void_p(), C.c_void_p(), C.c_void_p()
        self._check(self.lib.bwagpu_chain2aln_results_dense(self.ctx, slot, C.byref(rp), C.byref(np_), C.byref(op)),
                    "results_dense")
        nr = batch.n_reads
        if nr == 0:
            return np.zeros(0, abi.ALNREG_DTYPE), np.zeros(0, np.int32)
        cnt = np.ctypeslib.as_array(C.cast(np_, C.POINTER(C.c_int32)), (nr,))
        tot = int(np.ctypeslib.as_array(C.cast(op, C.POINTER(C.c_int32)), (nr + 1,))[nr])
        view = (np.ctypeslib.as_array(C.cast(rp, C.POINTER(C.c_uint8)), (tot * abi.ALNREG_DTYPE.itemsize,))
                .view(abi.ALNREG_DTYPE) if tot else np.zeros(0, abi.ALNREG_DTYPE))
        if out is None:
            return view, cnt
        regs, n = out
        if len(regs) < tot or len(n) < nr:
            raise ValueError("wait_dense: out arrays too small")
        n[:nr] = cnt
        regs[:tot] = view
        return regs[:tot], n[:nr]

    def chain2aln_device(self, dev_batch: abi.BatchC, dev_out: int, dev_n: int, dev_stats: int | None,
                         stream: int | None):
        self._check(self.lib.bwagpu_chain2aln_device(self.ctx, C.byref(dev_batch), C.c_void_p(dev_out),
                                                     C.c_void_p(dev_n),
                                                     C.c_void_p(dev_stats) if dev_stats else None,
                                                     C.c_void_p(stream) if stream else None),
                    "chain2aln_device")

    def extend_batch(self, tasks: np.ndarray, qpool: np.ndarray, tpool: np.ndarray) -> np.ndarray:
        tasks = np.ascontiguousarray(tasks, abi.EXT_TASK_DTYPE)
        qpool = np.ascontiguousarray(qpool, np.uint8)
        tpool = np.ascontiguousarray(tpool, np.uint8)
        res = np.zeros(max(len(tasks), 1), abi.EXT_RES_DTYPE)
        self._check(self.lib.bwagpu_extend_batch(self.ctx, len(tasks), _ptr(tasks), _ptr(qpool), len(qpool),
                                                 _ptr(tpool), len(tpool), _ptr(res)), "extend_batch")
        return res[:len(tasks)]

    def align2_batch(self, tasks: np.ndarray, qpool: np.ndarray, tpool: np.ndarray) -> np.ndarray:
        """ksw_align2 (bwa/ksw.c:337-357) per task -> kswr_t records (abi.KSWR_DTYPE)"""
        tasks = np.ascontiguousarray(tasks, abi.ALIGN2_TASK_DTYPE)
        qpool = np.ascontiguousarray(qpool, np.uint8)
        tpool = np.ascontiguousarray(tpool, np.uint8)
        res = np.zeros(max(len(tasks), 1), abi.KSWR_DTYPE)
        self._check(self.lib.bwagpu_align2_batch(self.ctx, len(tasks), _ptr(tasks), _ptr(qpool), len(qpool),
                                                 _ptr(tpool), len(tpool), _ptr(res)), "align2_batch")
        return res[:len(tasks)]

    def align2_device(self, n: int, dev_tasks: int, dev_q: int, dev_t: int, dev_out: int, dev_scratch: int,
                      stream: int | None = None):
        """asynchronous launch on device buffers (pointers as ints, e.g. torch data_ptr())"""
        self._check(self.lib.bwagpu_align2_device(self.ctx, n, dev_tasks, dev_q, dev_t, dev_out, dev_scratch,
                                                  stream), "align2_device")

    def reg2aln_batch(self, tasks: np.ndarray, qpool: np.ndarray, max_ops: int = 64, max_md: int = 512):
        """mem_reg2aln's CIGAR part (bwa/bwamem.c:1104-1174) per job -> (abi.ALN_DTYPE records,
        CIGAR ops [n, max_ops] uint32, MD strings [n, max_md] bytes)"""
        tasks = np.ascontiguousarray(tasks, abi.REG2ALN_TASK_DTYPE)
        qpool = np.ascontiguousarray(qpool, np.uint8)
        n = len(tasks)
        out = np.zeros(max(n, 1), abi.ALN_DTYPE)
        cig = np.zeros((max(n, 1), max_ops), np.uint32)
        md = np.zeros((max(n, 1), max_md), np.uint8)
        self._check(self.lib.bwagpu_reg2aln_batch(self.ctx, n, _ptr(tasks), _ptr(qpool), len(qpool), max_ops, max_md,
                                                  _ptr(out), _ptr(cig), _ptr(md)), "reg2aln_batch")
        return out[:n], cig[:n], md[:n]

    def set_bwt(self, hdr, words, sa=None, sa_intv: int = 32):
        """make the FM-index resident (hdr = primary, L2[0..4], seq_len as bwa's bwt_t;
        sa = the sampled suffix array, for bwt_sa)"""
        hdr = np.asarray(hdr, np.int64)
        self._bwt_words = np.ascontiguousarray(words, np.uint32)
        self._bwt_sa = None if sa is None else np.ascontiguousarray(sa, np.uint64)
        b = abi.BwtC()
        b.primary = int(hdr[0])
        for i in range(5):
            b.L2[i] = int(hdr[1 + i])
        b.seq_len = int(hdr[6])
        b.bwt_size = len(self._bwt_words)
        b.bwt = self._bwt_words.ctypes.data
        if self._bwt_sa is not None:
            b.sa_intv = sa_intv
            b.n_sa = len(self._bwt_sa)
            b.sa = self._bwt_sa.ctypes.data
        self._check(self.lib.bwagpu_set_bwt(self.ctx, C.byref(b)), "set_bwt")

    def bwt_sa(self, ks) -> np.ndarray:
        """bwt_sa (bwa/bwt.c:86-96) per BWT position"""
        ks = np.ascontiguousarray(ks, np.uint64)
        out = np.zeros(max(len(ks), 1), np.uint64)
        self._check(self.lib.bwagpu_bwt_sa(self.ctx, len(ks), _ptr(ks), _ptr(out)), "bwt_sa")
        return out[:len(ks)]

    def sw_stream(self, words: np.ndarray, cap_tasks: int) -> np.ndarray:
        """sw_top on the FPGA wire format (src/fpga/FPGAPipeline.cpp:252-336 in,
        :91-105 out): one packed task stream -> int16[n_tasks, 10] records"""
        words = np.ascontiguousarray(words, np.int32)
        out = np.zeros((max(cap_tasks, 1), 10), np.int16)
        n = C.c_int32(0)
        self._check(self.lib.bwagpu_sw_stream(self.ctx, _ptr(words), len(words), _ptr(out), int(cap_tasks),
                                              C.byref(n)), "sw_stream")
        return out[:n.value]

    # bwagpu_debug_ext_kernel codes -> the first bin's extension kernel
    EXT_KERNELS = {8: "spec_ext4_kernel<16, 10, true>", 4: "spec_ext4_kernel<32, 5, true>",
                   5: "spec_ext4_kernel<32, 8, false>", 2: "spec_ext2_kernel<5>",
                   # the phased pair: one "launch" = its left and right side launches
                   18: "spec_side4_kernel<16, 10, true>", 14: "spec_side4_kernel<32, 5, true>",
                   15: "spec_side4_kernel<32, 8, false>", 28: "spec_sidep_kernel<16, 10, true>"}

    def ext_kernel(self, lq_max: int = 256) -> str:
        """the first length bin's extension kernel this context launches for
        reads of up to lq_max bases (the C side's own decision, spec.hip
        ext_kernel_for)"""
        k = self.lib.bwagpu_debug_ext_kernel(self.ctx, int(lq_max))
        if k not in self.EXT_KERNELS:
            raise BwaGpuError(k, "debug_ext_kernel")
        return self.EXT_KERNELS[k]

    def ext_form(self, form: int = -1) -> int:
        """this context's extension form (bwagpu_ctx_ext_form); -> the previous one"""
        return self.lib.bwagpu_ctx_ext_form(self.ctx, int(form))

    def row_bound(self, on: int = -1) -> int:
        """this context's row bound in the packed extension kernels
        (bwagpu_ctx_row_bound, default on); -> the previous setting"""
        return self.lib.bwagpu_ctx_row_bound(self.ctx, int(on))

    def set_device_read_len(self, max_len: int):
        """bound on the read lengths of later device batches (bwagpu_set_device_read_len)"""
        self._check(self.lib.bwagpu_set_device_read_len(self.ctx, int(max_len)), "set_device_read_len")

    def sup_shift(self, shift: int):
        """superblock size 2^shift of the occurrence layout the NEXT set_bwt builds (tests; default 32)"""
        self._check(self.lib.bwagpu_debug_sup_shift(self.ctx, shift), "sup_shift")

    def seed_budget(self, budget: int):
        """bwt_extend calls a read gets on one lane before the wave kernel takes it (0: all on waves)"""
        self._check(self.lib.bwagpu_debug_seed_budget(self.ctx, budget), "seed_budget")

    def collect_intv(self, seq_off: np.ndarray, seq: np.ndarray, min_seed_len: int = 19, split_width: int = 10,
                     max_mem_intv: int = 20, split_factor: float = 1.5, max_per_read: int = 256,
                     out_cap: int | None = None, out: np.ndarray | None = None):
        """mem_collect_intv (bwa/bwamem.c:120-167) per read -> (counts int32[n], intervals INTV_DTYPE[sum]);
        out: the caller's INTV_DTYPE buffer to fill (reused across calls; its length is the capacity)"""
        seq_off = np.ascontiguousarray(seq_off, np.int64)
        seq = np.ascontiguousarray(seq, np.uint8)
        n = len(seq_off) - 1
        o = abi.SeedOpt(min_seed_len, split_width, max_mem_intv, split_factor)
        if out is not None:
            if out.dtype != abi.INTV_DTYPE or not out.flags.c_contiguous:
                raise ValueError("out must be a contiguous INTV_DTYPE array")
            cap = len(out)
        else:
            cap = max(n, 1) * max_per_read if out_cap is None else out_cap
            out = np.zeros(max(cap, 1), abi.INTV_DTYPE)
        cnt = np.zeros(max(n, 1), np.int32)
        self._check(self.lib.bwagpu_collect_intv(self.ctx, C.byref(o), n, _ptr(seq_off), _ptr(seq), max_per_read,
                                                 _ptr(out), cap, _ptr(cnt)), "collect_intv")
        cnt = cnt[:n]
        return cnt, out[:int(cnt.sum())]

    def set_alt(self, is_alt):
        """per-contig ALT flags for the chaining (None: none)"""
        self._alt = None if is_alt is None else np.ascontiguousarray(is_alt, np.uint8)
        self._check(self.lib.bwagpu_set_alt(self.ctx, None if self._alt is None else _ptr(self._alt)), "set_alt")

    @staticmethod
    def _seed_chain_opts(seedopt, split_factor, chainopt):
        so = np.asarray(seedopt, np.int32)
        co = abi.default_chainopt() if chainopt is None else chainopt
        return (abi.SeedOpt(int(so[0]), int(so[1]), int(so[2]), float(split_factor)),
                abi.ChainOpt(int(co["max_occ"]), int(co["max_chain_gap"]), int(co["min_chain_weight"]),
                             int(co["max_chain_extend"]), float(co["mask_level"]), float(co["drop_ratio"])))

    def seqs2chains(self, seq_off, seq, seedopt=(19, 10, 20), split_factor: float = 1.5, chainopt: dict | None = None,
                    raw: bool = False, copy: bool = True):
        """bwa-flow's SeqsToChains on the device (src/bwa_wrapper.cpp:105-115) ->
        (read_chain_off int32[n+1], chains CHAIN_DTYPE, chain_seed_off int32, seeds SEED_DTYPE);
        copy=False: views of the context's pinned output (valid until its next call)"""
        seq_off = np.ascontiguousarray(seq_off, np.int64)
        seq = np.ascontiguousarray(seq, np.uint8)
        n = len(seq_off) - 1
        so, co = self._seed_chain_opts(seedopt, split_factor, chainopt)
        out = abi.ChainsC()
        self._check(self.lib.bwagpu_seqs2chains(self.ctx, C.byref(so), C.byref(co), n, _ptr(seq_off), _ptr(seq),
                                                int(raw), C.byref(out)), "seqs2chains")
        nc, ns = out.n_chains, out.n_seeds

        def view(p, dt, k):
            if k == 0:
                return np.zeros(0, dt)
            v = np.frombuffer((C.c_char * (k * np.dtype(dt).itemsize)).from_address(p), dt)
            return v.copy() if copy else v
        return (view(out.read_chain_off, np.int32, n + 1), view(out.chains, abi.CHAIN_DTYPE, nc),
                view(out.chain_seed_off, np.int32, nc + 1), view(out.seeds, abi.SEED_DTYPE, ns))

    def seqs2regions(self, seq_off, seq, seedopt=(19, 10, 20), split_factor: float = 1.5,
                     chainopt: dict | None = None, copy: bool = True):
        """SeqsToChains + ChainsToRegions fused on the device -> (regions per read int32[n],
        regions ALNREG_DTYPE back to back in read order); copy=False: the regions as a
        view of the context's pinned output (valid until its next call)"""
        seq_off = np.ascontiguousarray(seq_off, np.int64)
        seq = np.ascontiguousarray(seq, np.uint8)
        n = len(seq_off) - 1
        so, co = self._seed_chain_opts(seedopt, split_factor, chainopt)
        cnt = np.zeros(max(n, 1), np.int32)
        regs, nreg = C.c_void_p(), C.c_int64()
        self._check(self.lib.bwagpu_seqs2regions(self.ctx, C.byref(so), C.byref(co), n, _ptr(seq_off), _ptr(seq),
                                                 _ptr(cnt), C.byref(regs), C.byref(nreg)), "seqs2regions")
        k = nreg.value
        out = np.zeros(0, abi.ALNREG_DTYPE) if k == 0 else np.frombuffer(
            (C.c_char * (k * abi.ALNREG_DTYPE.itemsize)).from_address(regs.value), abi.ALNREG_DTYPE)
        return cnt[:n], (out.copy() if copy else out)

    def prof_start(self, max_launches: int):
        """time the next max_launches launches of the dominant extension kernel"""
        self._check(self.lib.bwagpu_prof_start(self.ctx, max_launches), "prof_start")

    def prof_intervals(self, max_n: int = 4096):
        """-> float64[n, 2]: each timed launch's [start, end] in ms from the first event"""
        a = np.zeros(max(max_n, 1), np.float64)
        b = np.zeros(max(max_n, 1), np.float64)
        n = C.c_int32(0)
        self._check(self.lib.bwagpu_prof_intervals(self.ctx, _ptr(a), _ptr(b), int(max_n), C.byref(n)), "prof_intervals")
        return np.stack([a[:n.value], b[:n.value]], axis=1)

    def prof_read(self) -> tuple[float, int]:
        """-> (summed kernel ms, launches timed) since prof_start"""
        ms, n = C.c_double(), C.c_int32()
        self._check(self.lib.bwagpu_prof_read(self.ctx, C.byref(ms), C.byref(n)), "prof_read")
        return ms.value, n.value

    def last_stats(self, slot: int = 0) -> dict:
        s = abi.Stats()
        self._check(self.lib.bwagpu_last_stats(self.ctx, slot, C.byref(s)), "last_stats")
        return {k: getattr(s, k) for k, _ in abi.Stats._fields_}
