"""Drop-in for the reference's DistributedSamplerViaLocallyShuffleV2.py (V2, two pools).

    from partiallyshuffledistributedsampler_amd.DistributedSamplerViaLocallyShuffleV2 import \
        DistributedSamplerViaLocallyShuffle
"""
from .sampler import _PartialShuffleSampler


class DistributedSamplerViaLocallyShuffle(_PartialShuffleSampler):
    """V2: TensorFlow-style shuffle buffer (pool1 of shuffle_buffer slots refilled from
    pool2), emulated on the GPU in slot-replacement form (reference V2:96-116).  `shuffle`
    is accepted and ignored, as in the reference (V2:142-152)."""
    _VERSION = 2

    def _warm_msg(self):
        return str(self.rank) + ': warm start!!'
