"""MI355X-native partial-shuffle distributed sampler (drop-in for
microsoft/PartiallyShuffleDistributedSampler).  See DESIGN.md.

V1 / V2 samplers live in the modules named like the reference files:
    from partiallyshuffledistributedsampler_amd.DistributedSamplerViaLocallyShuffle import \
        DistributedSamplerViaLocallyShuffle            # one pool
    from partiallyshuffledistributedsampler_amd.DistributedSamplerViaLocallyShuffleV2 import \
        DistributedSamplerViaLocallyShuffle            # two pools
"""
__version__ = "0.1.0"


def __getattr__(name):
    if name in ("DistributedSamplerViaLocallyShuffle", "DistributedSamplerViaLocallyShuffleV1"):
        from .DistributedSamplerViaLocallyShuffle import DistributedSamplerViaLocallyShuffle
        return DistributedSamplerViaLocallyShuffle
    if name == "DistributedSamplerViaLocallyShuffleV2":
        from .DistributedSamplerViaLocallyShuffleV2 import DistributedSamplerViaLocallyShuffle
        return DistributedSamplerViaLocallyShuffle
    if name == "IndexEngine":
        from .engine import IndexEngine
        return IndexEngine
    raise AttributeError(name)
