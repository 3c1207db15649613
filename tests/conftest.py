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


def set_c2a_path(path, monkeypatch):
    """mem_chain2aln paths of the GPU tests:
      spec  the speculative extension tasks + selection passes, first two
            read-length bins with packed 16-bit DP (the default: eight seeds
            per wave in the first bin, four in the second)
      quad  the same with four seeds per wave in both bins (bwagpu_debug_ext_form(2))
      pair  the same with two seeds per wave (32-bit DP; bwagpu_debug_ext_form(1))
      fast  the per-read kernels (BWAGPU_C2A_PATH=fast: a wave per read), an
            independent implementation kept as a cross-check
    The form is the default of contexts created afterwards (bwagpu_debug_ext_form;
    bwagpu_ctx_ext_form sets one context's): restored by the caller's teardown."""
    from bwagpu import abi
    lib = abi.load()
    if path == "fast":
        monkeypatch.setenv("BWAGPU_C2A_PATH", "fast")
    else:
        monkeypatch.delenv("BWAGPU_C2A_PATH", raising=False)
    prev = lib.bwagpu_debug_ext_form({"pair": 1, "quad": 2}.get(path, 0))
    return lambda: lib.bwagpu_debug_ext_form(prev)
