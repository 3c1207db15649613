"""TEST INFRASTRUCTURE ONLY: packs oracle/_ref/gen_chain's output (the
reference's own mem_chain -> mem_chain_flt -> mem_flt_chained_seeds per read,
gen_chain.c) into tests/golden/chain_<set>.npz.

    make -C oracle ref && python oracle/gen_chain.py

The genome and FM-index are the golden ones (tests/golden/ref.npz,
seed_bwt.npz); this script checks that the generator's pac and occurrence
array equal them before writing anything.

chain_<set>.npz  reads (nt4) and, per read, mem_chain's raw chains (kbtree
                 traversal order: pos, rid, n, is_alt + seeds) and the chains
                 mem_chain_flt / mem_flt_chained_seeds leave (pos, rid, n, w,
                 kept, first, is_alt, frac_rep + seeds with scores)
"""
import hashlib
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "..", "tests", "golden")
SETS = [  # name, read seed, reads, lengths, opt mode, ALT contig, min raw chains
    ("c1", 51, 3000, "150", 0, -1, 0),
    ("mix", 53, 2000, "100,150,250,40,19,12", 0, 1, 0),
    ("long", 55, 600, "750,800,1000", 0, -1, 0),
    ("opt", 57, 2000, "150,250", 1, 2, 0),
    ("rep", 59, 600, "150,250", 0, -1, 6),
    ("longopt", 61, 300, "800,1000", 1, -1, 3),
]


def rd(d, name, dt):
    return np.fromfile(os.path.join(d, name + ".bin"), dt)


def main():
    exe = os.path.join(HERE, "_ref", "gen_chain")
    ref = np.load(os.path.join(GOLD, "ref.npz"))
    bwt = np.load(os.path.join(GOLD, "seed_bwt.npz"))
    for name, seed, n, lens, om, alt, mraw in SETS:
        with tempfile.TemporaryDirectory() as d:
            subprocess.run([exe, d, str(seed), str(n), lens, str(om), str(alt), str(mraw)], check=True)
            if not np.array_equal(rd(d, "pac", np.uint8), ref["pac"]):
                raise SystemExit("gen_chain's genome differs from tests/golden/ref.npz")
            if hashlib.sha256(rd(d, "bwt", np.uint32).tobytes()).digest() != \
                    hashlib.sha256(bwt["words"].tobytes()).digest():
                raise SystemExit("gen_chain's index differs from tests/golden/seed_bwt.npz")
            np.savez_compressed(
                os.path.join(GOLD, f"chain_{name}.npz"), opt=rd(d, "opt", np.int32), optf=rd(d, "optf", np.float32),
                alt_rid=np.array([alt], np.int32), seq_off=rd(d, "seq_off", np.int64), seq=rd(d, "seq", np.uint8),
                raw_n=rd(d, "raw_n", np.int32), raw_chn=rd(d, "raw_chn", np.int64).reshape(-1, 4),
                raw_seed=rd(d, "raw_seed", np.int64).reshape(-1, 3), chn_n=rd(d, "chn_n", np.int32),
                chn=rd(d, "chn", np.int64).reshape(-1, 7), chn_frac=rd(d, "chn_frac", np.float32),
                seed=rd(d, "seed", np.int64).reshape(-1, 4), stats=rd(d, "stats", np.int64))
            print(f"[gen_chain] chain_{name}: stats {rd(d, 'stats', np.int64).tolist()}")


if __name__ == "__main__":
    main()
