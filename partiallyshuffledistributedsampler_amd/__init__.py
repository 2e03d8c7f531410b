"""MI355X-native partial-shuffle distributed sampler (drop-in for
microsoft/PartiallyShuffleDistributedSampler).  See DESIGN.md."""
__version__ = "0.1.0"
