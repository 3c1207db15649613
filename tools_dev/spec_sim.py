"""CPU simulation of the speculative path's emulation against the reference's
own decisions: C2 batch 0's regions from the oracle
(in extension order) give, by replaying bwamem.c:676-715 on them, which seeds
the reference extends; the emulation (round-A regions only, pending seeds
optimistic) is replayed beside it.  Prints the round-A / round-B waste with a
cell-cost model (q * (q + min(q, w)) per side), then the two-phase round B
experiment for reads with > 32 seeds.

    python tools_dev/spec_sim.py
"""
import os, sys
REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [os.path.join(REPO, p) for p in ("bwa-flow_amd/python", "tests", "oracle")]
import numpy as np
from bwagpu import workload
import oracle as orc
opt, ref, bs = workload.load_fixture()
rb = bs[0]; b = rb.batch
R = orc.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
regs, n, st = orc.chain2aln("oracle", opt, R, b, 8)
lq = np.diff(b.seq_off); cso = b.chain_seed_off; rco = b.read_chain_off; S = b.seeds
def cal_max_gap(q):
    a=opt['a']; l_del = int((q*a - opt['o_del'])/opt['e_del'] + 1.); l_ins=int((q*a-opt['o_ins'])/opt['e_ins']+1.)
    l = max(l_del, l_ins); l = max(l,1); return min(l, opt['w']<<1)
def hit_test(s, av, L):
    for p in av:
        if s['rbeg'] < p['rb'] or s['rbeg']+s['len'] > p['re'] or s['qbeg'] < p['qb'] or s['qbeg']+s['len'] > p['qe']: continue
        if s['len'] - p['seedlen0'] > .1*L: continue
        qd = s['qbeg']-p['qb']; rdd = s['rbeg']-p['rb']; w = min(cal_max_gap(min(qd,rdd)), p['w'])
        if qd-rdd < w and rdd-qd < w: return True
        qd = p['qe']-(s['qbeg']+s['len']); rdd = p['re']-(s['rbeg']+s['len']); w = min(cal_max_gap(min(qd,rdd)), p['w'])
        if qd-rdd < w and rdd-qd < w: return True
    return False
def overlap_exc(sd, order, kk, srt, s):
    for i in order[:kk]:
        if srt[i] == 0: continue
        tt = sd[i]
        if tt['len'] < s['len']*.95: continue
        if s['qbeg'] <= tt['qbeg'] and s['qbeg']+s['len']-tt['qbeg'] >= s['len']>>2 and tt['qbeg']-s['qbeg'] != tt['rbeg']-s['rbeg']: return True
        if tt['qbeg'] <= s['qbeg'] and tt['qbeg']+tt['len']-s['qbeg'] >= s['len']>>2 and s['qbeg']-tt['qbeg'] != s['rbeg']-tt['rbeg']: return True
    return False
def pred_region(s, L, mode):
    if mode == 'full':
        return dict(rb=int(s['rbeg'])-int(s['qbeg']), re=int(s['rbeg'])+L-int(s['qbeg']), qb=0, qe=L, seedlen0=int(s['len']), w=opt['w'])
    if mode == 'seed':
        return dict(rb=int(s['rbeg']), re=int(s['rbeg'])+int(s['len']), qb=int(s['qbeg']), qe=int(s['qbeg'])+int(s['len']), seedlen0=int(s['len']), w=opt['w'])

# ---- waste by round (cost model)

NR = 66668
costA = costA_w = 0; nA_w = 0; costB = costB_w = 0; cost_ref = 0
def cost(L, s):
    ql = int(s['qbeg']); qr = L - ql - int(s['len'])
    # rows ~ q + min(q, w) ; width ~ q  -> cells ~ q*(q+min(q,100))
    return ql*(ql+min(ql,100)) + qr*(qr+min(qr,100))
heavyB_w = 0
for rd in range(NR):
    L = int(lq[rd]); c0, c1 = rco[rd], rco[rd+1]
    s0 = cso[c0]; av = regs[s0:s0+n[rd]]
    t = 0; truth = {}; avt = []
    for ch in range(c0, c1):
        sd = S[cso[ch]:cso[ch+1]]
        order = sorted(range(len(sd)), key=lambda i: (int(sd[i]['score']), i), reverse=True)
        srt = {i: 1 for i in order}
        for kk, k in enumerate(order):
            s = sd[k]
            if hit_test(s, avt, L) and not overlap_exc(sd, order, kk, srt, s):
                srt[k] = 0; continue
            if t < len(av): truth[(ch,k)] = av[t]; avt.append(av[t])
            t += 1
    ns = cso[c1]-cso[c0]
    ave = []; B = set()
    for ch in range(c0, c1):
        sd = S[cso[ch]:cso[ch+1]]
        order = sorted(range(len(sd)), key=lambda i: (int(sd[i]['score']), i), reverse=True)
        c = cost(L, sd[order[0]]); costA += c
        if (ch, order[0]) not in truth: costA_w += c; nA_w += 1
        srt = {i: 1 for i in order}
        for kk, k in enumerate(order):
            s = sd[k]
            if hit_test(s, ave, L) and not overlap_exc(sd, order, kk, srt, s):
                srt[k] = 0; continue
            if kk == 0:
                if (ch,k) in truth: ave.append(truth[(ch,k)])
            else:
                B.add((ch,k)); c = cost(L, s); costB += c
                if (ch,k) not in truth:
                    costB_w += c
                    if ns > 32: heavyB_w += c
    for (ch,k) in truth: cost_ref += cost(L, S[cso[ch]+k])
print("A cost", costA, "A waste", costA_w, nA_w, "B cost", costB, "B waste", costB_w, "heavy(ns>32) B waste", heavyB_w, "ref cost", cost_ref)
print("waste frac", (costA_w+costB_w)/(costA+costB))

# ---- two-phase round B for heavy reads

NR = 66668
def cost(L, s):
    ql = int(s['qbeg']); qr = L - ql - int(s['len'])
    return ql*(ql+min(ql,100)) + qr*(qr+min(qr,100))
def diag(s): return int(s['rbeg']) - int(s['qbeg'])
tot = dict(B=0, Bw=0, B1=0, B1w=0, B2=0, B2w=0, miss=0, costB=0, costBw=0, cost12=0, cost12w=0)
for rd in range(NR):
    L = int(lq[rd]); c0, c1 = rco[rd], rco[rd+1]
    s0 = cso[c0]; av = regs[s0:s0+n[rd]]
    t = 0; truth = {}; avt = []
    for ch in range(c0, c1):
        sd = S[cso[ch]:cso[ch+1]]
        order = sorted(range(len(sd)), key=lambda i: (int(sd[i]['score']), i), reverse=True)
        srt = {i: 1 for i in order}
        for kk, k in enumerate(order):
            s = sd[k]
            if hit_test(s, avt, L) and not overlap_exc(sd, order, kk, srt, s):
                srt[k] = 0; continue
            if t < len(av): truth[(ch,k)] = av[t]; avt.append(av[t])
            t += 1
    ns = cso[c1]-cso[c0]
    def emulate(known):   # known: set of B seeds whose true regions are available
        ave = []; B = []
        for ch in range(c0, c1):
            sd = S[cso[ch]:cso[ch+1]]
            order = sorted(range(len(sd)), key=lambda i: (int(sd[i]['score']), i), reverse=True)
            srt = {i: 1 for i in order}
            for kk, k in enumerate(order):
                s = sd[k]
                if hit_test(s, ave, L) and not overlap_exc(sd, order, kk, srt, s):
                    srt[k] = 0; continue
                if kk == 0:
                    if (ch,k) in truth: ave.append(truth[(ch,k)])
                elif (ch,k) in known:
                    if (ch,k) in truth: ave.append(truth[(ch,k)])
                else:
                    B.append((ch,k))
        return B
    B = emulate(set())
    tot['B'] += len(B); w = [x for x in B if x not in truth]; tot['Bw'] += len(w)
    cB = sum(cost(L, S[cso[ch]+k]) for ch,k in B); tot['costB'] += cB
    tot['costBw'] += sum(cost(L, S[cso[ch]+k]) for ch,k in w)
    if ns <= 32:
        tot['cost12'] += cB; tot['cost12w'] += sum(cost(L, S[cso[ch]+k]) for ch,k in w)
        continue
    # heavy: B1 = pending seeds with no earlier pending seed near their diagonal
    B1 = []; seen = []
    for ch,k in B:
        s = S[cso[ch]+k]; d = diag(s)
        if not any(abs(d - e) < 2*opt['w'] for e in seen): B1.append((ch,k))
        seen.append(d)
    B2 = emulate(set(B1))   # optimistic second emulation with B1's regions
    B2 = [x for x in B2 if x not in B1]
    allB = B1 + B2
    tot['B1'] += len(B1); tot['B1w'] += sum(1 for x in B1 if x not in truth)
    tot['B2'] += len(B2); tot['B2w'] += sum(1 for x in B2 if x not in truth)
    tot['cost12'] += sum(cost(L, S[cso[ch]+k]) for ch,k in allB)
    tot['cost12w'] += sum(cost(L, S[cso[ch]+k]) for ch,k in allB if (ch,k) not in truth)
print(tot)
