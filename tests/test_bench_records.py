"""Host logic of bench.py's profile lookups (no GPU): roofline.traffic and the rocprofv3 figures are
taken only from stamped records of the exact kernel symbol that ran and of the same config, preferring
the record made with the loaded library (then with its sources, then the newest stamp), never by
directory name; the builder's micro-benchmark ceilings from stamped records
(ceilings.json), the current tool code's first, then the newest."""
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


def _rec(d, config, kernels, lib="L0", src="S0", utc="2026-01-01T00:00:00Z", stamp=True):
    """kernels: {symbol: (avg_ns, hbm_bytes_per_launch)}"""
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "kernel_stats.csv"), "w") as f:
        f.write('"Name","Calls","TotalDurationNs","AverageNs"\n')
        for k, (ns, _) in kernels.items():
            f.write(f'"{k}",10,{10 * ns},{ns}\n')
    json.dump({"config": config, "kernels": {k: {"hbm_bytes_per_launch": b} for k, (_, b) in kernels.items()}},
              open(os.path.join(d, "pmc_summary.json"), "w"))
    if stamp:
        json.dump({"config": config, "lib_sha256": lib, "src_sha256": src, "utc": utc},
                  open(os.path.join(d, "stamp.json"), "w"))


def test_record_exact_symbol_config_and_stamp(bench, tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "_IDENT", {"lib": "LIB", "src": "SRC"})
    _rec(tmp_path / "zz_old", "cfg3", {SYM_BQ: (500.0, 222)}, utc="2026-01-01T00:00:00Z")
    _rec(tmp_path / "aa_new", "cfg3", {SYM_BQ: (400.0, 333)}, utc="2026-02-01T00:00:00Z")
    # newest stamp wins when no stamp matches the library (not the alphabetically last directory)
    r = bench.find_record("cfg3", SYM_BQ, str(tmp_path))
    assert (r["traffic_bytes_per_launch"], r["dir"], r["match"]) == (333, "profiles/aa_new", "none")
    assert r["avg_us"] == 0.4
    # a record of the same sources beats a newer one; one of the same library beats both
    _rec(tmp_path / "mm_src", "cfg3", {SYM_BQ: (450.0, 444)}, src="SRC", utc="2025-12-01T00:00:00Z")
    assert bench.find_record("cfg3", SYM_BQ, str(tmp_path))["match"] == "src"
    _rec(tmp_path / "bb_lib", "cfg3", {SYM_BQ: (420.0, 555)}, lib="LIB", utc="2025-11-01T00:00:00Z")
    r = bench.find_record("cfg3", SYM_BQ, str(tmp_path))
    assert (r["traffic_bytes_per_launch"], r["match"]) == (555, "lib")
    # another config, another symbol, a substring, no symbol, an unstamped directory: no record
    _rec(tmp_path / "cc_cfg4", "cfg4", {SYM_BQ: (900.0, 666)}, lib="LIB", utc="2027-01-01T00:00:00Z")
    assert bench.find_record("cfg3", SYM_BQ, str(tmp_path))["traffic_bytes_per_launch"] == 555
    assert bench.find_record("cfg4", SYM_BQ, str(tmp_path))["traffic_bytes_per_launch"] == 666
    assert bench.find_record("cfg3", SYM_B3, str(tmp_path)) is None
    assert bench.find_record("cfg3", "k_pass_bq", str(tmp_path)) is None
    assert bench.find_record("cfg3", None, str(tmp_path)) is None
    _rec(tmp_path / "dd_unstamped", "cfg3", {SYM_B3: (100.0, 1)}, stamp=False)
    assert bench.find_record("cfg3", SYM_B3, str(tmp_path)) is None


def _ceiling_rec(d, files, utc, tools=None):
    os.makedirs(d, exist_ok=True)
    for name, text in files.items():
        (d / name).write_text(text)
    if utc is not None:
        json.dump({"kind": "ceilings", "utc": utc, "tool_code_sha256": tools or {}}, open(d / "ceilings.json", "w"))


def test_ceilings_by_stamp(bench, tmp_path):
    """Micro-benchmark ceilings come from stamped records (ceilings.json), the current tool code's
    first, then the newest stamp -- never from a directory name or the round."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import stamp as st
    cur = {t: st.code_sha(os.path.join(ROOT, "tools", t)) for t in ("wrbench.hip", "aqbench.hip")}
    aq = "AQ rows (y, N - y), half lines"
    _ceiling_rec(tmp_path / "zz_unstamped", {"wrbench.txt": "write nt 192 MiB         grid  2048     43.5 us   4632.1 GB/s\n",
                                             "aqbench.txt": aq + "         17.2 us   7800.8 GB/s\n"}, None)
    assert bench.write_ceilings(str(tmp_path)) is None
    assert bench.shape_us("aqbench.txt", aq, str(tmp_path)) is None
    _ceiling_rec(tmp_path / "r02_old", {"wrbench.txt": "write nt 192 MiB         grid  2048     44.0 us   4600.0 GB/s\n"
                                                       "write nt 1 GiB           grid  4096    263.9 us   4069.1 GB/s\n",
                                        "aqbench.txt": aq + "         17.0 us   7900.0 GB/s\n"},
                 "2025-01-01T00:00:00Z", cur)
    wc = bench.write_ceilings(str(tmp_path))
    assert wc["nt_192MiB_GBs"] == 4600.0 and wc["nt_beyond_cache_GBs"] == 4069.1
    assert wc["source"] == "profiles/r02_old/wrbench.txt"
    assert bench.shape_us("aqbench.txt", aq, str(tmp_path))[0] == 17.0
    # newer, same code: wins; newer still but another tool code: loses to the current code's record
    _ceiling_rec(tmp_path / "aa_new", {"aqbench.txt": aq + "         16.5 us   8000.0 GB/s\n"}, "2025-06-01T00:00:00Z", cur)
    _ceiling_rec(tmp_path / "bb_other_code", {"aqbench.txt": aq + "         15.0 us   9000.0 GB/s\n"},
                 "2026-01-01T00:00:00Z", {"aqbench.hip": "0" * 64})
    assert bench.shape_us("aqbench.txt", aq, str(tmp_path)) == (16.5, "profiles/aa_new/aqbench.txt")
    # the committed tree quotes a stamped record
    assert bench.write_ceilings() is not None
    assert bench.shape_us("aqbench.txt", aq) is not None and bench.shape_us("bqbench.txt", "texture layout, nt") is not None


def test_mip_record_per_frame(bench, tmp_path, monkeypatch):
    """update_loop's mip kernels from the update_loop record: k_mips_block runs once per frame, so
    the per-frame time is the record's total mip time over the block kernel's launches."""
    monkeypatch.setattr(bench, "_IDENT", {"lib": "LIB", "src": "SRC"})
    blk = "ocean::(anonymous namespace)::k_mips_block(ocean::DevView, int, int)"
    tail = "ocean::(anonymous namespace)::k_mips_tail(ocean::DevView, int)"
    assert bench.mip_record(str(tmp_path)) is None
    _rec(tmp_path / "r04u", "update_loop", {blk: (30000.0, 1), tail: (6000.0, 1)}, lib="LIB")
    r = bench.mip_record(str(tmp_path))
    assert r["us_per_frame"] == 36.0 and r["match"] == "lib" and set(r["kernels"]) == {"k_mips_block", "k_mips_tail"}
    _rec(tmp_path / "r04c", "cfg3", {blk: (1.0, 1), tail: (1.0, 1)}, lib="LIB", utc="2027-01-01T00:00:00Z")
    assert bench.mip_record(str(tmp_path))["dir"] == "profiles/r04u"  # another config's record never stands in


def test_entry_record_sums_the_four_step_pair(bench, tmp_path, monkeypatch):
    """At N >= 2048 one timed column entry launches C1 then C2; the library names C2.  The entry's
    rocprofv3 time and PMC traffic are the two records summed (round 3 compared C2 alone with the
    entry's bytes, a 1.16 'fraction')."""
    monkeypatch.setattr(bench, "_IDENT", {"lib": "LIB", "src": "SRC"})
    c1 = "void ocean::(anonymous namespace)::k_col4s1<4096, true>(ocean::DevView, int)"
    c2 = "void ocean::(anonymous namespace)::k_col4s2<4096, 4, true>(ocean::DevView, int)"
    _rec(tmp_path / "r04c5", "cfg5", {c1: (84000.0, 470), c2: (130000.0, 739)}, lib="LIB")
    r = bench.entry_record("cfg5", c2, str(tmp_path))
    assert r["avg_us"] == 214.0 and r["traffic_bytes_per_launch"] == 1209 and r["kernels"] == [c1, c2]
    assert bench.entry_record("cfg5", SYM_BQ, str(tmp_path)) is None
    _rec(tmp_path / "r04c3", "cfg3", {SYM_BQ: (55000.0, 336)}, lib="LIB")
    r = bench.entry_record("cfg3", SYM_BQ, str(tmp_path))
    assert r["avg_us"] == 55.0 and r["kernels"] == [SYM_BQ]
    _rec(tmp_path / "r04c5b", "cfg5", {c2: (1.0, 1)}, lib="LIB", utc="2027-01-01T00:00:00Z")  # C2 alone, newer
    assert bench.entry_record("cfg5", c2, str(tmp_path)) is None  # the pair's records sit in two directories


def test_cfg1_line(bench):
    """BASELINE configs[0] has a bench line: `bench.py --config cfg1` runs the scalar
    CPU path at 256^2 x 1 with no GPU and prints one JSON line of the contract's keys, n_gpus 0, the
    path labelled as the C port standing in for the C# one."""
    import subprocess
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "cfg1", "--steps", "6",
                          "--warmup", "2"], capture_output=True, text=True, timeout=300, check=True).stdout
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "vs_baseline", "dtype", "data", "config", "path", "init_spectrum_ms"):
        assert k in d, k
    assert d["n_gpus"] == 0 and d["steps"] == 6 and d["unit"] == "frames/s" and d["value"] > 0
    assert d["config"]["workload"].startswith("cfg1") and d["config"]["n"] == 256 and d["config"]["cascades"] == 1
    assert d["path"]["kind"] == "port" and d["path"]["cores"] == 1 and "CpuOcean.cs" in d["path"]["what"]
