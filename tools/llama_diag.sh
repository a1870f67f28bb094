#!/bin/bash
# run each llama_diag configuration in its own process; stop at the first crash
set -e
run() { echo "== $*"; env "$@" 2>&1 | grep -v "^llama_\|^llama.cpp\|amdgpu.ids" ; }
run CFG=default timeout -k 10 120 python tools/llama_diag.py 4 2
run CFG=evals1 timeout -k 10 120 python tools/llama_diag.py 4 1
run CFG=threads1 timeout -k 10 120 python tools/llama_diag.py 1 1
run CFG=nocache GGML_HIP_WEIGHT_CACHE=0 timeout -k 10 120 python tools/llama_diag.py 4 1
run CFG=nommap REFLLAMA_NO_MMAP=1 timeout -k 10 120 python tools/llama_diag.py 4 1
run CFG=nopinned GGML_HIP_NO_PINNED=1 timeout -k 10 120 python tools/llama_diag.py 4 1
