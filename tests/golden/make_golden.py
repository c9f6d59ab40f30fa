"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py

The reference (Unity/HLSL) ships no golden vectors and cannot run here, so
these vectors come from oracle/ocean_oracle.c (the fp32 restatement of the
reference's kernels; see its header for file:line citations).  They pin the
oracle and the GPU path against regressions; the oracle itself is pinned by
the independent known-answer tests in tests/test_oracle.py.

Each case is one .npz (float32 arrays) plus an entry in manifest.json with the
inputs (params, cascades, seed, times) and the sha256 of the file.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

CASES = [
    # name, N, cascades (indices into SCENE_CASCADES), shallow, seed, times, nplanes
    ("scene_n32_c4_deep", 32, [0, 1, 2, 3], False, 20251121, [0.0, 1.25, 100.0], 4),
    ("scene_n16_c3_shallow", 16, [0, 1, 2], True, 20251122, [0.5, 1.0, 1.5], 4),
    ("scene_n64_c1_disp", 64, [0], False, 20251121, [1.25], 2),
]


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        h.update(f.read())
    return h.hexdigest()


def main():
    manifest = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/ocean_oracle.c", "cases": []}
    for name, n, cidx, shallow, seed, times, nplanes in CASES:
        params = O.scene_params(shallow)
        cascades = [O.SCENE_CASCADES[i] for i in cidx]
        noise = O.generate_noise(n, seed)
        oc = O.OracleOcean(n, params, cascades, noise, nplanes=nplanes)
        arrays = {"noise": noise, "h0": oc.h0, "waves": oc.waves}
        for f, t in enumerate(times):
            disp, deriv, turb = oc.step(t)
            arrays[f"disp_{f}"] = disp.copy()
            if nplanes == 4:
                arrays[f"deriv_{f}"] = deriv.copy()
                arrays[f"turb_{f}"] = turb.copy()
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **arrays)
        manifest["cases"].append(dict(name=name, file=name + ".npz", n=n, params=params, cascades=cascades,
                                      seed=seed, times=times, nplanes=nplanes, sha256=sha256(path)))
    # operator-level IFFT case: random complex planes, C=2, N=32
    rng = np.random.default_rng(7)
    plane = rng.standard_normal((2, 32, 32, 2)).astype(np.float32)
    out = O.ifft2d(plane)
    path = os.path.join(HERE, "ifft_n32_c2.npz")
    np.savez_compressed(path, input=plane, output=out)
    manifest["cases"].append(dict(name="ifft_n32_c2", file="ifft_n32_c2.npz", n=32, sha256=sha256(path),
                                  note="IFFT.InverseFastFourierTransform on a random float2[2][32][32] array"))
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", [c["file"] for c in manifest["cases"]])


if __name__ == "__main__":
    main()
