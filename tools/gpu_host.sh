#!/bin/bash
# host-prologue change check: full -m gpu suite, C2 bench at N=1, 2-process same-GPU rehearsal
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/host; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-latency > $O/c2.json 2> $O/c2.err
PSS_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-latency > $O/rehearse_c2.json 2> $O/rehearse_c2.err
nproc > $O/nproc.txt
python - > $O/prologue.txt <<'PY'
import time, sys
import numpy as np
sys.path.insert(0, ".")
import workloads as W
from partiallyshuffledistributedsampler_amd.engine import IndexEngine
l1, N1, R1, B, _ = W.shape("c2")
for world in (1, 4, 8):
    lengths = np.tile(l1, world)
    eng = IndexEngine(lengths, int(lengths.sum()), R1 * world, B, 2, seed=0, device="cpu")
    for e in range(5):
        eng.init_iter(e)
    t = time.perf_counter()
    for e in range(5, 105):
        eng.init_iter(e)
    print("world", world, "init_iter back to back ms %.4f" % ((time.perf_counter() - t) / 100 * 1e3))
    eng.close()
PY
echo done
