"""ldagibbssampling_amd — MI355X-native collapsed-Gibbs LDA sampler.

Drop-in for the hot path of qianjinding/LDAGibbsSampling: the per-token
z-resampling loop that the reference reaches through Mallet 2.0.7's
ParallelTopicModel.estimate() (src/cmu_ron/TrainAndPredict.java:159-171,
src/cmu/TrainAndPredict.java:258-269).  Compute runs in hand-written HIP
kernels for gfx950 behind the C ABI in include/lda_mi355x.h.
"""
from .capi import LdaError, MAX_TOPICS, padded_topics  # noqa: F401
from .corpus import Corpus  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # Lazily import the GPU-facing classes so that the CPU-only parts
    # (corpus formats, build) import without the HIP library.
    if name == "GibbsSampler":
        from .sampler import GibbsSampler
        return GibbsSampler
    if name in ("ParallelTopicModel", "TopicInferencer", "InstanceList"):
        from . import topic_model
        return getattr(topic_model, name)
    raise AttributeError(name)
