"""Test helpers: import path of the product binding + GPU availability."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "llama.cpp-q_4_0_amd")
sys.path.insert(0, os.path.join(PKG, "python"))

import ggml_hip  # noqa: E402

LIB_PATH = ggml_hip.LIB_PATH


def gpu_available():
    try:
        return os.path.exists(LIB_PATH) and ggml_hip.device_count() > 0
    except Exception:
        return False
