"""Loader for the golden fixtures in tests/golden (generated from the reference by tools/gen_golden.py)."""
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names(prefix=""):
    out = []
    for f in sorted(os.listdir(GOLDEN)):
        if f.endswith(".npz") and f.startswith(prefix) and not f.startswith("init_"):
            out.append(f[:-4])
    return out


def split(flat, shapes, dtype=np.float32):
    out, k = [], 0
    for s in shapes:
        n = int(np.prod(s))
        out.append(np.asarray(flat[k:k + n], dtype=dtype).reshape(s))
        k += n
    return out


def load(name):
    """A fixture with its factor lists split; float64 fixtures (f64_*) keep float64 inputs."""
    d = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    meta = json.loads(str(d.pop("meta")))
    shapes = [tuple(s) for s in meta["factor_shapes"]]
    dt = np.float64 if meta.get("model") == "linear_f64" else np.float32
    d["X"] = _x_of(d, dt)
    d["Bcp0_list"] = split(d["Bcp0"], shapes, dt)
    if "Bcp_final" in d:
        d["Bcp_final_list"] = split(d["Bcp_final"], shapes, dt)
    if "grads0" in d:
        d["grads0_list"] = split(d["grads0"], shapes, dt)
    if "Bcp_10" in d:
        d["Bcp_10_list"] = split(d["Bcp_10"], shapes, dt)
    if "Bcp_final2" in d:
        d["Bcp_final2_list"] = split(d["Bcp_final2"], shapes, dt)
    d["meta"] = meta
    d["shapes"] = shapes
    return d


def _x_of(d, dt):
    """X of a fixture: int8 / 8 (exact in fp32 and in bf16), or stored as float32 (X_f32:
    full-mantissa inputs, the *_f32x fixtures)."""
    if "X_f32" in d:
        return torch.tensor(d["X_f32"].astype(dt))
    return torch.tensor(d["X_q"].astype(dt) / 8.0)


def normwise_rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.linalg.norm(b.ravel())
    return float(np.linalg.norm((a - b).ravel()) / (den if den > 0 else 1.0))


def load_spectral(name):
    """Spectral fixture: factor lists Bcp_n (I, Rn, 1) and Bcp_c (W, Rs, Cc), (D, Rs, 1), (n_out, Rs, 1)."""
    d = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    meta = json.loads(str(d.pop("meta")))
    sn = [tuple(s) for s in meta["factor_shapes_n"]]
    sc = [tuple(s) for s in meta["factor_shapes_c"]]
    d["X"] = _x_of(d, np.float32)
    for key in ("Bcp_n0", "Bcp_n_10", "Bcp_n_final", "grads_n0"):
        if key in d:
            d[key + "_list"] = split(d[key], sn) if d[key].size else [np.zeros(s, np.float32) for s in sn]
    for key in ("Bcp_c0", "Bcp_c_10", "Bcp_c_final", "grads_c0"):
        if key in d:
            d[key + "_list"] = split(d[key], sc) if d[key].size else [np.zeros(s, np.float32) for s in sc]
    d["meta"] = meta
    d["shapes_n"], d["shapes_c"] = sn, sc
    return d
