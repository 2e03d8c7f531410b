"""The BASELINE.json configurations as synthetic inputs.

Shared by bench.py, tools/bench_configs.py and the tests so that every one of them measures
or checks exactly the same shapes.  Each entry gives the files_len array (dataset order),
num_replicas, shuffle_buffer and sampler version; nothing here touches the GPU.

  c1  V1 on CPU: 64 files x 10,000 samples, R = 2, B = 4096          (BASELINE configs[0])
  c2  V2: 10,000 files x 10,000 = 100M samples, R = 8, B = 4096      (configs[1])
  c3  V2: 100,000 files x 10,000 = 1B samples, R = 1024, B = 4096    (configs[2], 128 ranks/GPU)
  c4  V2: Zipf(1.5) * 150 file sizes, F = 100,000 (N = 2,594,705,250 > 2^31), R = 4096
                                                                      (configs[3])
  c5  V2: c2's files, B = 2^20 (pools beyond LDS), R = 8, epochs 0..99 (configs[4])
"""
import numpy as np

# name: (description, files, samples per file or "zipf", R, B, version)
CONFIGS = {
    "c1": ("V1 one-pool sampler, 64 files x 10K samples, R=2, B=4096 (CPU plumbing config)",
           64, 10_000, 2, 4096, 1),
    "c2": ("V2 two-pool sampler, 10K files x 10K samples = 100M, R=8, B=4096",
           10_000, 10_000, 8, 4096, 2),
    "c3": ("V2, 100K files x 10K samples = 1B, R=1024 logical ranks (128 per GPU at 8 GPUs), B=4096",
           100_000, 10_000, 1024, 4096, 2),
    "c4": ("V2, Zipf(1.5)*150 file sizes over 100K files (N=2,594,705,250), R=4096, B=4096",
           100_000, "zipf", 4096, 4096, 2),
    "c5": ("V2, 10K files x 10K = 100M, R=8, B=2^20 (pools beyond LDS), per-epoch reseed",
           10_000, 10_000, 8, 1 << 20, 2),
}


def lengths(name):
    """files_len of a configuration, in dataset order (int64)."""
    _, F, L, _, _, _ = CONFIGS[name]
    if L == "zipf":
        z = np.random.default_rng(0).zipf(1.5, F) * 150
        return np.clip(z, 1, 2_000_000).astype(np.int64)
    return np.full(F, L, dtype=np.int64)


def shape(name):
    """(lengths, N, R, B, version) of a configuration."""
    _, _, _, R, B, ver = CONFIGS[name]
    ln = lengths(name)
    return ln, int(ln.sum()), R, B, ver
