"""moss_tts_amd -- MI355X-native (gfx950 / CDNA4) engine for the MossTTSDelay decode path.

Drop-in for `moss_tts_delay.modeling_moss_tts.MossTTSDelayModel.generate` and the
processor I/O surface (xiami2019/MOSS-TTS).  Compute runs in hand-written HIP
kernels (csrc/) behind the C ABI of include/mtts.h; PyTorch is used for weight
loading and device memory only.
"""
__version__ = "0.1.0"
