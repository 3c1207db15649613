"""The speculative path's A/B knobs,
each in a child process of its own (the library reads BWAGPU_* once per
process): round 5's emulation (no round-B task for an uncertain skip: the
final pass extends misses inline, round C runs for the long reads), the task
state machine instead of the phased extension, both length bins phased, the
producer-wave kernel, the risky-first final pass.  Every variant must give the
reference's regions, byte for byte, on the C2 fixture's batches and the C5
fixture's mixed-length batch.  One child at a time."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))

VARIANTS = {
    "emu_strict_off": {"BWAGPU_EMU_STRICT": "0"},
    "task_state_machine": {"BWAGPU_EXT_PHASED": "0"},
    "both_bins_phased": {"BWAGPU_EXT_PHASED": "3"},
    "producer_waves": {"BWAGPU_EXT_PRODUCER": "1"},
    "risky_first": {"BWAGPU_LIGHT_RISKY_FIRST": "1"},
}


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_variant_parity(name):
    env = dict(os.environ, **VARIANTS[name])
    p = subprocess.run([sys.executable, os.path.join(HERE, "gpu_variant_child.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["c2"] and all(r["c2"]), r
    assert r["c5"] and all(r["c5"]), r
