import sys, ctypes
sys.path.insert(0, "/root/repo")
import numpy as np
from partiallyshuffledistributedsampler_amd.engine import IndexEngine
from partiallyshuffledistributedsampler_amd import _lib
lengths = np.full(10, 1000)
eng = IndexEngine(lengths, 10000, 2, 100, 2, device=0)
print("emit path auto ->", eng.emit_path())
