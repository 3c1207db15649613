#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY — regenerate tests/golden/*.npz from the reference.

Runs oracle/_ref/gen_golden (the reference's own bwa C: index, seeding,
chaining, mem_chain2aln, ksw_extend2 — see gen_golden.c) and the reference
ksw_extend2 on randomised edge-case tasks (via oracle/_ref/libbwaref.so), and
packs inputs + reference outputs as numpy .npz fixtures (no pickles).

    make -C oracle && python oracle/gen_golden.py
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.normpath(os.path.join(HERE, ".."))
GOLD = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, HERE)
import oracle  # noqa: E402
from oracle import abi  # noqa: E402

RTASK = np.dtype([("qlen", "<i4"), ("tlen", "<i4"), ("w", "<i4"), ("end_bonus", "<i4"), ("zdrop", "<i4"),
                  ("h0", "<i4"), ("qoff", "<i8"), ("toff", "<i8")])

# name -> (read seed, pairs, read-length mode, opt mode)
CHAIN_SETS = {
    "c1_default": (42, 1000, "150", 0),
    "c5_mixed": (7, 450, "mix", 0),
    "opt1_scoring": (11, 400, "150", 1),
    "opt2_band": (13, 400, "150", 2),
}
N_TASKS_KEEP = 1200


def rd(d, name, dt):
    return np.fromfile(os.path.join(d, name + ".bin"), dtype=dt)


def subsample_tasks(tasks, res, qpool, tpool, n, rng):
    idx = np.sort(rng.choice(len(tasks), size=min(n, len(tasks)), replace=False))
    out_t = np.zeros(len(idx), abi.EXT_TASK_DTYPE)
    qs, ts, qo, to = [], [], 0, 0
    for k, i in enumerate(idx):
        t = tasks[i]
        qs.append(qpool[t["qoff"]:t["qoff"] + t["qlen"]])
        ts.append(tpool[t["toff"]:t["toff"] + t["tlen"]])
        out_t[k] = (qo, to, t["qlen"], t["tlen"], t["w"], t["end_bonus"], t["zdrop"], t["h0"])
        qo += int(t["qlen"])
        to += int(t["tlen"])
    r = np.zeros(len(idx), abi.EXT_RES_DTYPE)
    for f in abi.EXT_RES_DTYPE.names:
        r[f] = res[f][idx]
    return out_t, r, np.concatenate(qs).astype(np.uint8), np.concatenate(ts).astype(np.uint8)


def gen_chain_set(name, seed, pairs, lm, om, tmp, rng):
    d = os.path.join(tmp, name)
    os.makedirs(d, exist_ok=True)
    subprocess.run([os.path.join(HERE, "_ref", "gen_golden"), d, str(seed), str(pairs), lm, str(om)], check=True)
    oi = rd(d, "opt_int", np.int32)
    opt = dict(zip(["a", "b", "o_del", "e_del", "o_ins", "e_ins", "pen_clip5", "pen_clip3", "w", "zdrop"],
                   oi.tolist()))
    mat = rd(d, "opt_mat", np.int8)
    ref = dict(l_pac=rd(d, "l_pac", np.int64), ann_offset=rd(d, "ann_offset", np.int64),
               ann_len=rd(d, "ann_len", np.int32), pac=rd(d, "pac", np.uint8))
    tasks = rd(d, "tasks", RTASK)
    res = rd(d, "task_res", abi.EXT_RES_DTYPE)
    t2, r2, q2, tp2 = subsample_tasks(tasks, res, rd(d, "qpool", np.uint8), rd(d, "tpool", np.uint8),
                                      N_TASKS_KEEP, rng)
    np.savez_compressed(
        os.path.join(GOLD, name + ".npz"),
        opt_int=oi, opt_mat=mat,
        seq_off=rd(d, "seq_off", np.int64), seq=rd(d, "seq", np.uint8),
        read_chain_off=rd(d, "read_chain_off", np.int32), chain_seed_off=rd(d, "chain_seed_off", np.int32),
        chain_rid=rd(d, "chain_rid", np.int32), chain_frac_rep=rd(d, "chain_frac_rep", np.float32),
        seeds=rd(d, "seeds", abi.SEED_DTYPE), reg_n=rd(d, "reg_n", np.int32), regs=rd(d, "regs", abi.ALNREG_DTYPE),
        tasks=t2, task_res=r2, qpool=q2, tpool=tp2)
    print(f"[gen_golden] {name}: reads={len(rd(d, 'seq_off', np.int64)) - 1} regions={len(rd(d, 'regs', abi.ALNREG_DTYPE))} "
          f"tasks kept={len(t2)}/{len(tasks)}")
    return opt, mat, ref


def edge_tasks(rng, n, allow_t5):
    """randomised ksw_extend2 calls covering the corners of ksw.c:380-479"""
    tasks = np.zeros(n, abi.EXT_TASK_DTYPE)
    qs, ts, qo, to = [], [], 0, 0
    special_q = [0, 1, 2, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 159, 160, 161, 255, 256, 257, 511, 700, 1022]
    for k in range(n):
        u = rng.random()
        if u < 0.25:
            ql = int(rng.choice(special_q))
        elif u < 0.8:
            ql = int(rng.integers(1, 160))
        else:
            ql = int(rng.integers(1, 300))
        q = rng.integers(0, 4, ql).astype(np.uint8)
        if rng.random() < 0.3 and ql:
            q[rng.random(ql) < 0.03] = 4
        mode = rng.random()
        if mode < 0.15:
            tl = int(rng.integers(0, 4))
            t = rng.integers(0, 4, tl).astype(np.uint8)
        elif mode < 0.3:
            tl = int(rng.integers(0, 400))
            t = rng.integers(0, 4, tl).astype(np.uint8)
        else:  # a diverged copy of the query, with indels and a random tail
            t = []
            for b in q:
                x = rng.random()
                if x < 0.02:
                    continue
                if x < 0.04:
                    t.extend(rng.integers(0, 4, int(rng.integers(1, 4))).tolist())
                t.append(int(rng.integers(0, 4)) if (b == 4 or rng.random() < 0.03) else int(b))
            t.extend(rng.integers(0, 4, int(rng.integers(0, 120))).tolist())
            if rng.random() < 0.15 and len(t) > 20:  # a junk middle triggers z-drop
                a = int(rng.integers(5, len(t) - 5))
                t[a:a + 40] = rng.integers(0, 4, 40).tolist()
            t = np.array(t, np.uint8)
            tl = len(t)
        if allow_t5 and tl and rng.random() < 0.2:
            t[rng.random(tl) < 0.05] = 4
        w = int(rng.choice([1, 2, 5, 10, 30, 100, 200, 300]))
        zd = int(rng.choice([0, 0, 5, 20, 100, 200]))
        eb = int(rng.integers(0, 11))
        h0 = int(rng.choice([1, 2, 5, 19, 30, 60, 150, 300]))
        tasks[k] = (qo, to, ql, tl, w, eb, zd, h0)
        qs.append(q)
        ts.append(t)
        qo += ql
        to += tl
    return tasks, np.concatenate(qs).astype(np.uint8), np.concatenate(ts).astype(np.uint8)


ALIGN2_OPTS = {
    "default": None,  # abi.default_opt()
    "scoring": dict(a=2, b=5, o_del=7, e_del=2, o_ins=5, e_ins=3, pen_clip5=3, pen_clip3=9, w=30, zdrop=40),
    # cheap gaps: an insertion next to a deletion beats a mismatch, so the
    # striped first pass (E from segment-local F) and the lazy-F early exit
    # of ksw_u8/ksw_i16 (o_ins == 0: equality case) decide the results
    "cheapgap": dict(a=5, b=12, o_del=1, e_del=1, o_ins=0, e_ins=1, pen_clip5=0, pen_clip3=0, w=50, zdrop=60),
    "cheapdel": dict(a=2, b=9, o_del=0, e_del=2, o_ins=1, e_ins=1, pen_clip5=0, pen_clip3=0, w=50, zdrop=60),
}
A2_SHORT = (1, 2, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129, 150, 200, 249, 250, 251, 255, 256, 300)


def gen_align2(rng):
    """ksw_align2 (mate rescue, bwamem_pair.c:150) through the reference's own code"""
    from bwagpu import synth
    for name, o in ALIGN2_OPTS.items():
        opt = abi.default_opt() if o is None else dict(o, mat=abi.fill_scmat(o["a"], o["b"]))
        parts = [synth.mate_rescue_tasks(rng, 250, a=opt["a"], qlens=(100, 150, 250), xtra_mode="matesw"),
                 synth.mate_rescue_tasks(rng, 250, a=opt["a"], qlens=A2_SHORT, win=(0, 400), xtra_mode="mix"),
                 synth.mate_rescue_tasks(rng, 40, a=opt["a"], qlens=(400, 700, 1023), win=(0, 900),
                                         xtra_mode="mix")]
        ts, qs, tps, qo, to = [], [], [], 0, 0
        for t, q, tp in parts:
            t = t.copy()
            t["qoff"] += qo
            t["toff"] += to
            ts.append(t); qs.append(q); tps.append(tp)
            qo += len(q); to += len(tp)
        tasks, qp, tp = np.concatenate(ts), np.concatenate(qs), np.concatenate(tps)
        res, _ = oracle.align2("ref", opt, tasks, qp, tp)
        np.savez_compressed(os.path.join(GOLD, "align2_" + name + ".npz"),
                            opt_int=np.array([opt[k] for k in ("a", "b", "o_del", "e_del", "o_ins", "e_ins",
                                                               "pen_clip5", "pen_clip3", "w", "zdrop")], np.int32),
                            opt_mat=np.asarray(opt["mat"], np.int8), tasks=tasks, task_res=res, qpool=qp, tpool=tp)
        print(f"[gen_golden] align2_{name}: tasks={len(tasks)} q={len(qp)} t={len(tp)} "
              f"tb>=0:{int((res['tb'] >= 0).sum())} score2>=0:{int((res['score2'] >= 0).sum())} "
              f"sat255:{int((res['score'] == 255).sum())}")


CTASK = np.dtype([("rb", "<i8"), ("re", "<i8"), ("qoff", "<i8"), ("l_seq", "<i4"), ("qb", "<i4"), ("qe", "<i4"),
                  ("truesc", "<i4"), ("w", "<i4"), ("read", "<i4")])
CRES = np.dtype([("pos", "<i8"), ("rid", "<i4"), ("is_rev", "<i4"), ("n_cigar", "<i4"), ("NM", "<i4"),
                 ("cig_off", "<i4"), ("md_off", "<i4"), ("md_len", "<i4"), ("pad", "<i4")])
CCALL = np.dtype([("task", "<i4"), ("w", "<i4"), ("l_query", "<i4"), ("score", "<i4"), ("n_cigar", "<i4"),
                  ("NM", "<i4"), ("cig_off", "<i4"), ("md_off", "<i4"), ("rb", "<i8"), ("re", "<i8")])


def gen_cigar(tmp):
    """mem_reg2aln (bwamem.c:1104-1174) on every region of each chain set, through
    the reference's own code (gen_golden records its outputs and every
    bwa_gen_cigar2 call) -> tests/golden/cigar_<set>.npz"""
    for name, (seed, pairs, lm, om) in CHAIN_SETS.items():
        d = os.path.join(tmp, "cig_" + name)
        os.makedirs(d, exist_ok=True)
        subprocess.run([os.path.join(HERE, "_ref", "gen_golden"), d, str(seed), str(pairs), lm, str(om)], check=True)
        ct, cr, cc = rd(d, "cig_tasks", CTASK), rd(d, "cig_res", CRES), rd(d, "cig_calls", CCALL)
        ops, md = rd(d, "cig_ops", np.uint32), rd(d, "cig_md", np.uint8)
        tasks = np.zeros(len(ct), abi.REG2ALN_TASK_DTYPE)
        for f in ("rb", "re", "qoff", "l_seq", "qb", "qe", "truesc", "w"):
            tasks[f] = ct[f]
        exp = np.zeros(len(ct), abi.ALN_DTYPE)
        for f in ("pos", "rid", "is_rev", "n_cigar", "NM", "md_len"):
            exp[f] = cr[f]
        last = np.full(len(ct), -1, np.int64)  # each job's last bwa_gen_cigar2 call: its score and band
        last[cc["task"]] = np.arange(len(cc))
        assert (last >= 0).all()
        exp["score"] = cc["score"][last]
        exp["w"] = cc["w"][last]
        np.savez_compressed(
            os.path.join(GOLD, "cigar_" + name + ".npz"),
            opt_int=rd(d, "opt_int", np.int32), opt_mat=rd(d, "opt_mat", np.int8),
            seq_off=rd(d, "seq_off", np.int64), seq=rd(d, "seq", np.uint8),
            tasks=tasks, exp=exp, cig_off=cr["cig_off"], md_off=cr["md_off"], cig_ops=ops, md=md,
            calls=cc)
        print(f"[gen_golden] cigar_{name}: jobs={len(ct)} gen_cigar2 calls={len(cc)} "
              f"multi-try jobs={int((np.bincount(cc['task'], minlength=len(ct)) > 1).sum())}")


def main():
    if "--only-align2" in sys.argv:
        gen_align2(np.random.default_rng(2025))
        return
    if "--only-cigar" in sys.argv:
        with tempfile.TemporaryDirectory() as tmp:
            gen_cigar(tmp)
        return
    if oracle.ref_lib() is None or not os.path.exists(os.path.join(HERE, "_ref", "gen_golden")):
        sys.exit("build the reference first: make -C oracle")
    os.makedirs(GOLD, exist_ok=True)
    rng = np.random.default_rng(2024)
    with tempfile.TemporaryDirectory() as tmp:
        ref = None
        for name, (seed, pairs, lm, om) in CHAIN_SETS.items():
            _, _, ref = gen_chain_set(name, seed, pairs, lm, om, tmp, rng)
        np.savez_compressed(os.path.join(GOLD, "ref.npz"), **ref)
        gen_cigar(tmp)
    # ksw_extend2 edge cases through the reference's own ksw_extend2
    opts = {
        "ksw_edge_default": abi.default_opt(),
        "ksw_edge_scoring": dict(a=2, b=5, o_del=7, e_del=2, o_ins=5, e_ins=3, pen_clip5=3, pen_clip3=9, w=30,
                                 zdrop=40, mat=abi.fill_scmat(2, 5)),
        "ksw_edge_matrix": dict(a=3, b=2, o_del=4, e_del=1, o_ins=9, e_ins=2, pen_clip5=0, pen_clip3=0, w=50,
                                zdrop=60, mat=np.array([3, -2, -1, -2, -1, -2, 2, -2, -1, 0, -1, -2, 4, -3, -2,
                                                        -2, -1, -3, 3, -1, -1, 0, -2, -1, 1], np.int8)),
    }
    for name, opt in opts.items():
        tasks, qp, tp = edge_tasks(rng, 1500, allow_t5=True)
        res, _ = oracle.extend("ref", opt, tasks, qp, tp)
        np.savez_compressed(os.path.join(GOLD, name + ".npz"),
                            opt_int=np.array([opt[k] for k in ("a", "b", "o_del", "e_del", "o_ins", "e_ins",
                                                               "pen_clip5", "pen_clip3", "w", "zdrop")], np.int32),
                            opt_mat=np.asarray(opt["mat"], np.int8), tasks=tasks, task_res=res, qpool=qp, tpool=tp)
        print(f"[gen_golden] {name}: tasks={len(tasks)} q={len(qp)} t={len(tp)}")
    gen_align2(np.random.default_rng(2025))


if __name__ == "__main__":
    main()
