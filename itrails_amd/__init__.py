"""itrails_amd — MI355X-native decoding core for the iTRAILS coalescent HMM.

Drop-in for the per-column hot path of trails-phylogeny/itrails: the forward /
posterior / Viterbi sweeps over MAF blocks (itrails_amd.hmm, mirroring optimizer.py) and the
CTMC matrix-exponential model build (itrails_amd.model, itrails_amd.dense), computed by
hand-written HIP kernels for gfx950 behind the C ABI of include/itrails_hip.h (libitrails_hip.so, built in-tree).
"""
__version__ = "0.1.0"
