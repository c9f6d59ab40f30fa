"""The compiled C++ host (ocean-simulation_amd/host/abi_host, built by __graft_entry__.build())
walks the reference's WaterBody lifecycle through the C ABI -- Awake, Update with a readback
request every frame, GetWaterHeight, OnValidate, SampleWorld, OnDisable (WaterBody.cs:195-309)
-- as a non-Python host binds the library.  Every number it writes is checked against the
same sequence through the Python binding (bit-exact) and the displacement against the oracle."""
import json
import os
import subprocess

import numpy as np
import pytest

import ocean_hip as oh
import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("require_gpu")]

HOST = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ocean-simulation_amd", "host",
                    "abi_host")


def scene(n_cascades):
    return [dict(wavelength=c["wavelength"], cutoff_low=c["cutoff_low"], cutoff_high=c["cutoff_high"],
                 swell=c["swell"], fade=c["fade"]) for c in O.SCENE_CASCADES[:n_cascades]]


@pytest.mark.parametrize("n,C,F,mode", [(256, 3, 6, "height"), (256, 3, 6, "rgba"), (1024, 4, 4, "height"),
                                        (1024, 4, 4, "rgba"), (1024, 1, 20, "height")])  # 20 > the 4 queued requests
def test_cpp_host_lifecycle(tmp_path, n, C, F, mode):
    """mode: the facade's readback (water_body.h Readback): DISP.y alone (ocean_read_height_async, the
    default) or the RGBA slice; buoyancyData is [n][n] or [n][n][4], GetWaterHeight the same .g either way."""
    assert os.path.exists(HOST), "build it: make -C ocean-simulation_amd (or __graft_entry__.build())"
    env = dict(os.environ)
    r = subprocess.run([HOST, str(tmp_path), str(n), str(C), str(F), mode], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert summary["requested"] == F + 1 and summary["completed"] == F + 1  # one request per frame (:288)

    def load(name, shape):
        return np.fromfile(os.path.join(tmp_path, name), np.float32).reshape(shape)

    cas = scene(C)
    ctx = oh.OceanContext(n, C, 1, oh.F_MIPS)
    ctx.set_params(O.scene_params(), cas)
    ctx.generate_noise(42)
    ctx.init_spectrum()
    frames = []
    for f in range(F):
        ctx.step(f / 60.0)
        frames.append(ctx.read(oh.TEX_DISP, 0, 0))
    shape = (n, n) if mode == "height" else (n, n, 4)

    def buoy(disp):  # what buoyancyData holds for a landed RGBA slice
        return disp[..., 1] if mode == "height" else disp

    np.testing.assert_array_equal(load("buoyancy0.bin", shape), buoy(frames[-1]))
    # GetWaterHeight after Update f reads the newest completed request: frame k <= f, or 0 before any
    probes = [(0.0, 0.0), (-n / 2, -n / 2), (n / 2 - 1, 50.0), (500.0, -500.0)]
    heights = load("heights.bin", (F, 4))

    def at(disp, wx, wz):
        u = min(max((wx + n // 2) / n, 0.0), 1.0)
        v = min(max((wz + n // 2) / n, 0.0), 1.0)
        x, y = min(max(int(np.float32(u) * n), 0), n - 1), min(max(int(np.float32(v) * n), 0), n - 1)
        return disp[y, x, 1]  # buoyancyData[y * width + x].g (WaterBody.cs:202-208)

    last = -1
    for f in range(F):
        cands = [k for k in range(f + 1) if all(heights[f, i] == at(frames[k], *probes[i]) for i in range(4))]
        if not cands:
            assert not heights[f].any(), f"frame {f}: heights match no completed frame"
            continue
        assert max(cands) >= last
        last = max(cands)
    # OnValidate: staged params become active at the re-init, foam carried over
    windy = dict(O.scene_params(), wind_speed=12.0)
    ctx.set_params(windy, cas)
    ctx.init_spectrum()
    ctx.step(0.5)
    b1 = load("buoyancy1.bin", shape)
    np.testing.assert_array_equal(b1, buoy(ctx.read(oh.TEX_DISP, 0, 0)))
    disp, _, _ = O.OracleOcean(n, windy, cas, O.generate_noise(n, 42)).step(0.5)
    if mode == "height":
        assert O.rel_err(b1, disp[0, ..., 1]) <= 1e-5
    else:
        for ch in range(3):
            assert O.rel_err(b1[..., ch], disp[0, ..., ch]) <= 1e-5
    pts = np.array([[-300.0 + 97.5 * i, 40.0 - 13.25 * i, 0.5 * i] for i in range(8)], np.float32)
    np.testing.assert_array_equal(load("sample.bin", (8, 3, 4)), ctx.sample_world(pts))
    ctx.close()
