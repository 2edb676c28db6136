from .conv import (ConvSpec, conv3x3, feature_dtype, nchw_to_nhwc, nhwc_to_nchw, pad8, res_block, to_nhwc)
from .layout import pixel_shuffle, pixel_unshuffle

__all__ = ['ConvSpec', 'conv3x3', 'feature_dtype', 'nchw_to_nhwc', 'nhwc_to_nchw', 'pad8', 'res_block', 'to_nhwc',
           'pixel_shuffle', 'pixel_unshuffle']
