"""Which build of the engine a measurement belongs to.

source_digest() hashes the engine's sources (bwa-flow_amd/csrc/*.hip|h and
include/*.h) — the GPU box gets the tree without .git, so the PMC summaries
under profiles/ are tagged with this digest by the script that makes them
(tools_dev/pmc_traffic.py), and bench.py takes roofline.traffic only from a
summary of the SAME sources."""
from __future__ import annotations

import glob
import hashlib
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.normpath(os.path.join(HERE, "..", ".."))
REPO_ROOT = os.path.normpath(os.path.join(PKG_ROOT, ".."))


def source_digest() -> str:
    files = sorted(glob.glob(os.path.join(PKG_ROOT, "csrc", "*.hip")) + glob.glob(os.path.join(PKG_ROOT, "csrc", "*.h"))
                   + glob.glob(os.path.join(REPO_ROOT, "include", "*.h")))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode() + b"\0")
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]
