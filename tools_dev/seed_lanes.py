"""Per-lane stamps of tier 1 (BWAGPU_SEED_DBG, with BWAGPU_SEED_STEP=1: the
one-extension-per-step kernel writes them): extensions, pass-1 extensions and
wall_clock64 start/end per lane (100 MHz), for the last collect_intv call
in the file.  usage: python tools_dev/seed_lanes.py <dbg file> <n_reads>"""
import sys

import numpy as np

d = np.fromfile(sys.argv[1], dtype=np.int64)
n = int(sys.argv[2])
d = d[-8 * n:].reshape(2 * n, 4)
ext, steps, t0, t1 = d.T
live = t1 > 0
base = t0[live].min()
t0 = (t0 - base) / 100.0  # us
t1 = (t1 - base) / 100.0
dur = t1 - t0
print("kernel span %.1f us; lanes %d" % (t1[live].max(), live.sum()))
for name, sel in (("smem lanes", slice(0, n)), ("last-like lanes", slice(n, 2 * n))):
    e = ext[sel]
    s = steps[sel]
    du = dur[sel]
    print("%s: ext mean %.1f p50 %d p90 %d p99 %d max %d; pass-1 ext mean %.1f max %d; dur mean %.1f p99 %.1f max %.1f us"
          % (name, e.mean(), np.percentile(e, 50), np.percentile(e, 90), np.percentile(e, 99), e.max(), s.mean(),
             s.max(), du.mean(), np.percentile(du, 99), du.max()))
    big = e > 200
    if big.any():
        print("   us per extension on lanes with > 200: mean %.2f" % (du[big] / e[big]).mean())
nw = (2 * n + 63) // 64
wmax_ext = np.array([ext[64 * w:64 * w + 64].max() for w in range(nw)])
wsum_ext = np.array([ext[64 * w:64 * w + 64].sum() for w in range(nw)])
wstart = np.array([t0[64 * w:64 * w + 64].min() for w in range(nw)])
wend = np.array([t1[64 * w:64 * w + 64].max() for w in range(nw)])
wsteps = np.array([steps[64 * w:64 * w + 64].max() for w in range(nw)])
wd = wend - wstart
print("waves %d: duration mean %.1f p50 %.1f p99 %.1f max %.1f us; start max %.1f us"
      % (nw, wd.mean(), np.percentile(wd, 50), np.percentile(wd, 99), wd.max(), wstart.max()))
o = np.argsort(-wend)[:10]
for w in o:
    print("  wave %5d start %7.1f end %7.1f  max ext %5d  max steps %5d  sum ext %6d  us/step %.2f"
          % (w, wstart[w], wend[w], wmax_ext[w], wsteps[w], wsum_ext[w], wd[w] / max(1, wsteps[w])))
c = np.corrcoef(wd, wmax_ext)[0, 1]
print("corr(wave duration, max ext) %.2f; us per max-step overall %.2f" % (c, (wd / np.maximum(1, wsteps)).mean()))
