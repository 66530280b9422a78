"""MI355X-native MIL-NCE video-text contrastive pretraining (S3D-G + word2vec text tower).

Capabilities of KoDohwan/MIL-NCE_HowTo100M, re-designed for gfx950: NDHWC bf16 activations,
hand-written HIP/CDNA4 kernels for the hot ops (``csrc/``), RCCL over xGMI for data parallel
training with cross-GPU negatives.
"""
__version__ = "0.1.0"
