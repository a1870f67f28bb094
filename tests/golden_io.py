"""Loader for tests/golden/ fixtures (generated from the compiled reference by
tests/golden/gen_golden.c via `make -C oracle golden`)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_DT = {"u8": np.uint8, "f32": np.float32, "i64": np.int64}


def manifest(variant):
    with open(os.path.join(GOLDEN, f"{variant}_manifest.json")) as f:
        return json.load(f)


def load(variant, name):
    m = manifest(variant)[f"{variant}_{name}"]
    a = np.fromfile(os.path.join(GOLDEN, m["file"]), dtype=_DT[m["dtype"]])
    return a.reshape(m["shape"])
