"""CPU tests of the C ABI's device rule (ocean.h "Conventions", ABI 3+): every call makes its context's
device current for its own span and restores the caller's current device before it returns.

The driver's GPU box has one GPU, so the restore branch never runs there (every context is on the
caller's device).  Here the rule's implementation (ocean-simulation_amd/csrc/device_scope.h, the class
the library instantiates over hipGetDevice / hipSetDevice) runs over a two-device stub runtime through
the WaterBody lifecycle's entry points (tests/device_scope_test.cpp): caller on 1 with the context on 0,
the reverse, the same device, a refused switch and nested calls.  The test also checks that it would
catch a broken scope (mutants of the header must fail it), and that every entry point of ocean_abi.cpp
that touches the device enters through the scope."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ocean-simulation_amd", "csrc")
HEADER = os.path.join(CSRC, "device_scope.h")
TEST_SRC = os.path.join(ROOT, "tests", "device_scope_test.cpp")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def build_and_run(tmp_path, header_text, name):
    inc = tmp_path / name
    inc.mkdir()
    (inc / "device_scope.h").write_text(header_text)
    exe = tmp_path / (name + ".bin")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", str(inc), TEST_SRC, "-o", str(exe)],
                   check=True, capture_output=True, text=True, timeout=120)
    return subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)


def test_device_scope_over_two_device_stub(tmp_path):
    r = build_and_run(tmp_path, open(HEADER).read(), "real")
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr


# Each mutant breaks one rule of the scope; the stub test must fail on every one of them.
MUTANTS = {
    "no_restore": ("if (restore_) (void)Api::set(prev_);", ""),
    "restore_to_context_device": ("restore_ = prev_ >= 0;", "restore_ = prev_ >= 0; prev_ = device;"),
    "never_restore": ("restore_ = prev_ >= 0;", "restore_ = false;"),
    "set_even_when_current": ("if (prev_ == device) return;", ""),
    "restore_after_refused_switch": ("error_ = e;  // the caller's device is still current: nothing to restore",
                                     "error_ = e;\n            restore_ = true;"),
}


@pytest.mark.parametrize("mutant", sorted(MUTANTS))
def test_stub_test_catches_broken_scope(tmp_path, mutant):
    old, new = MUTANTS[mutant]
    text = open(HEADER).read()
    assert old in text, f"mutant {mutant} no longer applies to device_scope.h"
    r = build_and_run(tmp_path, text.replace(old, new), mutant)
    assert r.returncode != 0 and "FAIL" in r.stdout, f"mutant {mutant} survived:\n{r.stdout}"


def _entry_bodies():
    src = open(os.path.join(CSRC, "ocean_abi.cpp")).read()
    hdr = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "ocean", "ocean.h")).read(), flags=re.S)
    names = sorted(set(re.findall(r"\b(ocean_[a-z0-9_]+)\s*\(", hdr)))
    bodies = {}
    for name in names:
        m = re.search(r"^[a-z][\w\s\*]*\b" + name + r"\([^;{]*\)\s*\{", src, flags=re.M)
        assert m, f"{name} declared in ocean.h but not defined in ocean_abi.cpp"
        i, depth = m.end(), 1
        while depth:
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            i += 1
        bodies[name] = src[m.end():i]
    return bodies


# What puts work on, or allocates on, a device: any HIP call except the event queries (events carry their
# device) and pinned host memory (no device), a kernel launch, or the library's step / timing helpers.
DEVICE_WORK = re.compile(r"\bhip(?!Event(?:Query|Synchronize|ElapsedTime)\b|Host(?:Malloc|Free)\b)[A-Z]\w*\(|\blaunch|\bstep_\w+\(|"
                         r"\bfold_pending\(|\bread_impl\(|\bwrite_impl\(")


def test_every_device_entry_enters_through_the_scope():
    bodies = _entry_bodies()
    assert len(bodies) >= 38
    scoped = 0
    for name, body in bodies.items():
        in_scope = "OCEAN_ENTER(" in body or "DeviceScope " in body
        if DEVICE_WORK.search(body) or in_scope:
            assert in_scope, f"{name} touches the device outside the scope"
            scoped += 1
    assert scoped >= 25, scoped
