"""TEST INFRASTRUCTURE ONLY: packs oracle/_ref/gen_seed's output (the reference's
own bwt_smem1 / bwt_seed_strategy1 / ks_introsort_mem_intv driven by
mem_collect_intv's control flow, gen_seed.c) into tests/golden/seed_*.npz.

    make -C oracle ref && python oracle/gen_seed.py

seed_bwt.npz     the golden genome's BWT (bwa index of oracle/sim.h's genome,
                 1 Mbp, seed 1234): header + interleaved occurrence words,
                 the sampled suffix array, and the reference's bwt_sa on
                 20 010 BWT positions
seed_<set>.npz   reads (nt4, with N runs) and their intervals per read, in
                 the order mem_collect_intv leaves them (sorted by info)
"""
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "..", "tests", "golden")
SETS = [  # name, read seed, reads, lengths, N fraction
    ("c1", 41, 3000, "150", 0.001),
    ("mix", 43, 3000, "mix", 0.01),
]


def rd(d, name, dt):
    return np.fromfile(os.path.join(d, name + ".bin"), dt)


def main():
    exe = os.path.join(HERE, "_ref", "gen_seed")
    bwt_done = False
    for name, seed, n, lm, nf in SETS:
        with tempfile.TemporaryDirectory() as d:
            subprocess.run([exe, d, str(seed), str(n), lm, "1000000", str(nf)], check=True)
            if not bwt_done:
                np.savez_compressed(os.path.join(GOLD, "seed_bwt.npz"), hdr=rd(d, "bwt_hdr", np.int64),
                                    words=rd(d, "bwt", np.uint32), sa_hdr=rd(d, "sa_hdr", np.int64),
                                    sa=rd(d, "sa", np.uint64), sa_q=rd(d, "sa_q", np.uint64),
                                    sa_v=rd(d, "sa_v", np.uint64))
                bwt_done = True
            np.savez_compressed(os.path.join(GOLD, f"seed_{name}.npz"), opt=rd(d, "opt", np.int32),
                                split_factor=rd(d, "split_factor", np.float32), seq_off=rd(d, "seq_off", np.int64),
                                seq=rd(d, "seq", np.uint8), intv_n=rd(d, "intv_n", np.int32),
                                intv=rd(d, "intv", np.uint64).reshape(-1, 4))
            print(f"[gen_seed] seed_{name}: reads={n} intervals={int(rd(d, 'intv_n', np.int32).sum())}")


if __name__ == "__main__":
    main()
