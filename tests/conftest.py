"""pytest configuration: the `gpu` marker and import paths.

CPU tests (-m "not gpu") check the oracle against the reference's golden
vectors, the host logic and the C-ABI library's exports; GPU tests (-m gpu)
are the parity tests proper and go through the C ABI on an MI355X."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "bwa-flow_amd", "python"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950)")
