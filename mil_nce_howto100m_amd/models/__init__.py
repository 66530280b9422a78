from .s3dg import S3D, STConv3D, InceptionBlock, SelfGating, ALL_BLOCKS, INCEPTION_CFG
from .text import SentenceEmbedding

__all__ = ["S3D", "STConv3D", "InceptionBlock", "SelfGating", "SentenceEmbedding", "ALL_BLOCKS",
           "INCEPTION_CFG"]
