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


CIGAR_SETS = ["cigar_" + n for n in CHAIN_SETS]


def load_cigar_set(name):
    """mem_reg2aln jobs of one chain set -> opt, tasks, qpool (the reads), expected
    records, expected CIGAR ops per job, expected MD bytes per job"""
    z = _npz(name)
    exp = z["exp"].astype(abi.ALN_DTYPE)
    ops = [z["cig_ops"][o:o + n] for o, n in zip(z["cig_off"], exp["n_cigar"])]
    mds = [bytes(z["md"][o:o + n]) for o, n in zip(z["md_off"], exp["md_len"])]
    return opt_of(z), z["tasks"].astype(abi.REG2ALN_TASK_DTYPE), z["seq"], exp, ops, mds


def aln_mismatch(tasks, got, cig, md, exp, ops, mds, fields=("pos", "rid", "is_rev", "n_cigar", "NM", "md_len",
                                                                "score", "w", "status")) -> str | None:
    """bit-exact comparison of reg2aln outputs (records + CIGAR + MD) with expected ones"""
    bad = []
    for k in range(len(tasks)):
        why = [f for f in fields if got[f][k] != exp[f][k]]
        if not why and got["status"][k] == abi.ALN_OK:
            n = int(exp["n_cigar"][k])
            if not np.array_equal(cig[k, :n], ops[k]):
                why.append("cigar")
            if bytes(md[k, :int(exp["md_len"][k])]) != mds[k]:
                why.append("MD")
        if why:
            bad.append((k, why))
    if not bad:
        return None
    k, why = bad[0]
    return f"{len(bad)}/{len(tasks)} jobs differ; first #{k} {tasks[k]} in {why}: got {got[k]} want {exp[k]}"


def aln_expected_from(out, cig, md):
    """(records, ops list, md list) in the form aln_mismatch takes as expected"""
    ops = [cig[k, :int(out["n_cigar"][k])] for k in range(len(out))]
    mds = [bytes(md[k, :int(out["md_len"][k])]) for k in range(len(out))]
    return out, ops, mds


def synth_reg2aln_jobs(rng, ref_pac, l_pac, ann_offset, ann_len, n, lens=(100, 150, 250), mat=None):
    """mem_reg2aln jobs around real alignments of a synthetic reference: each
    read is a mutated copy (substitutions, 1-6 bp indels, N bases) of a window
    on either strand inside one contig; the region is the true window with
    jittered ends, a clipped query range, a local score that sometimes
    exceeds the global one (band doubling) and a random region band w"""
    def base(x):
        return (int(ref_pac[x >> 2]) >> ((~x & 3) << 1)) & 3

    tasks = np.zeros(n, abi.REG2ALN_TASK_DTYPE)
    qs, qo = [], 0
    for k in range(n):
        L = int(rng.choice(lens))
        c = int(rng.integers(0, len(ann_offset)))
        span = L + 40
        p0 = int(ann_offset[c]) + int(rng.integers(0, int(ann_len[c]) - span))
        win = [base(p0 + i) for i in range(span)]
        rev = bool(rng.random() < 0.5)
        read = []
        i = 20
        while len(read) < L and i < span:
            u = rng.random()
            if u < 0.01:
                i += int(rng.integers(1, 7))  # deletion in the read
                continue
            if u < 0.02:
                read.extend(rng.integers(0, 4, int(rng.integers(1, 7))).tolist())  # insertion
            b = win[i]
            read.append(4 if rng.random() < 0.003 else (int(rng.integers(0, 4)) if rng.random() < 0.02 else b))
            i += 1
        read = read[:L]
        L = len(read)
        ref_end = i
        qb = int(rng.integers(0, 6)) if rng.random() < 0.3 else 0
        qe = L - (int(rng.integers(0, 6)) if rng.random() < 0.3 else 0)
        rb = p0 + 20 + int(rng.integers(-3, 4)) + qb
        re = p0 + ref_end + int(rng.integers(-3, 4)) - (L - qe)
        if re <= rb:
            re = rb + 1
        if rev:  # the read is the reverse complement; the region lives on the reverse strand
            read = [3 - b if b < 4 else 4 for b in read[::-1]]
            qb, qe = L - qe, L - qb
            rb, re = 2 * l_pac - re, 2 * l_pac - rb
        a = 1 if mat is None else int(mat[0])
        truesc = int((qe - qb) * a * rng.choice([0.6, 0.9, 1.0, 1.3]))
        w = int(rng.choice([1, 5, 20, 100, 200]))
        tasks[k] = (rb, re, qo, L, qb, qe, truesc, w, 0)
        qs.append(np.array(read, np.uint8))
        qo += L
    return tasks, np.concatenate(qs)


SEED_SETS = ["c1", "mix"]


def load_seed_bwt():
    """-> (hdr int64[8]: primary, L2[0..4], seq_len, bwt_size; occurrence words uint32)"""
    z = _npz("seed_bwt")
    return z["hdr"], z["words"]


def load_seed_set(name):
    """-> (opt int32[3]: min_seed_len, split_width, max_mem_intv; split_factor; seq_off; seq;
    expected counts per read; expected intervals uint64[sum, 4] = x0, x1, x2, info)"""
    z = _npz("seed_" + name)
    return z["opt"], float(z["split_factor"][0]), z["seq_off"], z["seq"], z["intv_n"], z["intv"]


def load_seed_sa():
    """-> (sa_intv, sampled suffix array uint64, query BWT positions, the reference's bwt_sa of each)"""
    z = _npz("seed_bwt")
    return int(z["sa_hdr"][0]), z["sa"], z["sa_q"], z["sa_v"]


CHAIN_GOLD_SETS = ["c1", "mix", "long", "opt", "rep", "longopt"]


def load_chain_gold(name):
    """tests/golden/chain_<name>.npz (oracle/gen_chain.py: the reference's own mem_chain ->
    mem_chain_flt -> mem_flt_chained_seeds) -> dict with opt (bwagpu_opt_t dict), copt
    (bwagpu_chainopt_t dict), seedopt int32[3], split_factor, is_alt uint8[3], seq_off, seq,
    raw (rco, chains[pos, rid, n, is_alt], seeds[rbeg, qbeg, len]) and final
    (rco, chains[pos, rid, n, w, kept, first, is_alt], frac float32, seeds[rbeg, qbeg, len, score])"""
    z = _npz("chain_" + name)
    ov, fv = z["opt"], z["optf"]
    opt = dict(a=int(ov[6]), b=int(ov[7]), o_del=int(ov[8]), e_del=int(ov[9]), o_ins=int(ov[10]),
               e_ins=int(ov[11]), pen_clip5=5, pen_clip3=5, w=int(ov[0]), zdrop=100)
    opt["mat"] = abi.fill_scmat(opt["a"], opt["b"])
    copt = dict(max_occ=int(ov[2]), max_chain_gap=int(ov[1]), min_chain_weight=int(ov[3]),
                max_chain_extend=int(ov[4]), mask_level=float(fv[0]), drop_ratio=float(fv[1]))
    seedopt = np.array([ov[5], ov[12], ov[13]], np.int32)
    alt = np.zeros(3, np.uint8)
    if int(z["alt_rid"][0]) >= 0:
        alt[int(z["alt_rid"][0])] = 1
    return dict(opt=opt, copt=copt, seedopt=seedopt, split_factor=float(fv[2]), is_alt=alt,
                seq_off=z["seq_off"], seq=z["seq"],
                raw=(np.concatenate([[0], np.cumsum(z["raw_n"])]), z["raw_chn"], z["raw_seed"]),
                final=(np.concatenate([[0], np.cumsum(z["chn_n"])]), z["chn"], z["chn_frac"], z["seed"]))
