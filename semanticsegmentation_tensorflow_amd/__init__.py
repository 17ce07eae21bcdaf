"""MI355X-native (gfx950) training path for the conv encoder-decoder
segmentation models of SeunghwanByun/SemanticSegmentation_Tensorflow.

Host code mirrors the reference's TF1 call surface; all arithmetic runs in
hand-written HIP kernels behind the C-ABI of `include/segkern.h`.
"""
__version__ = "0.1.0"
