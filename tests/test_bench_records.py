"""Host logic of bench.py's profile lookups (no GPU): roofline.traffic and the rocprofv3 figures are
taken only from records of the exact kernel symbol that ran, and the builder's
micro-benchmark ceilings only from this round's profiles/<ROUND>* directories."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    pytest.importorskip("torch")
    sys.path.insert(0, ROOT)
    import bench as b
    return b


SYM_BQ = "void ocean::(anonymous namespace)::k_pass_bq<1024, false, 0>(ocean::DevView, int)"
SYM_B3 = "void ocean::(anonymous namespace)::k_pass_b3<1024, false, 0>(ocean::DevView, int)"


def _pmc(d, config, kernels):
    os.makedirs(d, exist_ok=True)
    json.dump({"config": config, "kernels": {k: {"hbm_bytes_per_launch": v} for k, v in kernels.items()}},
              open(os.path.join(d, "pmc_summary.json"), "w"))


def test_pmc_traffic_exact_symbol_and_config(bench, tmp_path):
    _pmc(tmp_path / "r02a", "cfg3", {SYM_B3: 111, SYM_BQ: 222})
    _pmc(tmp_path / "r03a", "cfg3", {SYM_B3: 333})       # newer, but only the stale kernel
    _pmc(tmp_path / "r03b", "cfg4", {SYM_BQ: 444})       # the kernel, but another config
    assert bench.pmc_traffic(SYM_BQ, "cfg3", str(tmp_path)) == (222, "r02a")
    assert bench.pmc_traffic(SYM_BQ, "cfg4", str(tmp_path)) == (444, "r03b")
    assert bench.pmc_traffic(SYM_B3.replace("1024", "512"), "cfg3", str(tmp_path)) is None
    # a substring of the symbol is not a match
    assert bench.pmc_traffic("k_pass_bq", "cfg3", str(tmp_path)) is None
    assert bench.pmc_traffic(None, "cfg3", str(tmp_path)) is None


def test_rocprof_kernel_us_exact_symbol(bench, tmp_path):
    d = tmp_path / "r03x"
    os.makedirs(d)
    with open(d / "ifft_kernel_stats.csv", "w") as f:
        f.write('"Name","Calls","TotalDurationNs","AverageNs"\n')
        f.write(f'"{SYM_B3}",10,1000,100.0\n"{SYM_BQ}",10,5000,500.0\n')
    assert bench.rocprof_kernel_us("ifft_kernel_stats.csv", SYM_BQ, str(tmp_path)) == (
        0.5, "profiles/r03x/ifft_kernel_stats.csv")
    assert bench.rocprof_kernel_us("ifft_kernel_stats.csv", "k_pass", str(tmp_path)) is None


def test_ceilings_only_from_this_round(bench, tmp_path):
    old = tmp_path / "r02x"
    os.makedirs(old)
    (old / "wrbench.txt").write_text("write nt 192 MiB         grid  2048     43.5 us   4632.1 GB/s\n")
    (old / "aqbench.txt").write_text("AQ rows (y, N - y), half lines         17.2 us   7800.8 GB/s\n")
    assert bench.write_ceilings(str(tmp_path)) is None
    assert bench.shape_us("aqbench.txt", "AQ rows (y, N - y), half lines", str(tmp_path)) is None
    cur = tmp_path / (bench.ROUND + "z")
    os.makedirs(cur)
    (cur / "wrbench.txt").write_text("write nt 192 MiB         grid  2048     44.0 us   4600.0 GB/s\n"
                                     "write nt 1 GiB           grid  4096    263.9 us   4069.1 GB/s\n")
    (cur / "aqbench.txt").write_text("AQ rows (y, N - y), half lines         17.0 us   7900.0 GB/s\n")
    wc = bench.write_ceilings(str(tmp_path))
    assert wc["nt_192MiB_GBs"] == 4600.0 and wc["nt_beyond_cache_GBs"] == 4069.1
    assert bench.shape_us("aqbench.txt", "AQ rows (y, N - y), half lines", str(tmp_path))[0] == 17.0
