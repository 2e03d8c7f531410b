"""Drop-in for the reference's DistributedSamplerViaLocallyShuffle.py (V1, one pool).

    from partiallyshuffledistributedsampler_amd.DistributedSamplerViaLocallyShuffle import \
        DistributedSamplerViaLocallyShuffle
"""
from .sampler import _PartialShuffleSampler


class DistributedSamplerViaLocallyShuffle(_PartialShuffleSampler):
    """V1: each rank's block is cut into shuffle_buffer-sized pools, each pool permuted
    independently on the GPU (reference V1:157-172)."""
    _VERSION = 1
