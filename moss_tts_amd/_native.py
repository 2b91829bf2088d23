"""ctypes binding of libmtts.so (the C ABI in include/mtts.h).

There is no fallback: if the HIP library is missing or fails to load, every
entry point raises.  Error codes map to the exceptions the reference raises
(ValueError for bad shapes, `modeling_moss_tts.py:253-254`; RuntimeError for
runtime failures).
"""
import ctypes
import os

_DEFAULT_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libmtts.so")
_LIB_PATH = os.environ.get("MTTS_LIB") or _DEFAULT_LIB

MTTS_OK = 0
MTTS_E_INVALID = -1
MTTS_E_OOM = -2
MTTS_E_HIP = -3
MTTS_E_UNSUPPORTED = -4
MTTS_E_PSE_TIMEOUT = -5


class MttsConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("hidden", "layers", "n_heads", "n_kv", "head_dim", "inter", "vocab",
                                            "n_vq", "audio_vocab")] + \
               [("rope_theta", ctypes.c_float), ("rms_eps", ctypes.c_float)] + \
               [(n, ctypes.c_int) for n in ("pad_token_id", "im_start_token_id", "im_end_token_id",
                                            "audio_start_token_id", "audio_end_token_id",
                                            "audio_user_slot_token_id", "audio_assistant_gen_slot_token_id",
                                            "audio_assistant_delay_slot_token_id", "audio_pad_code",
                                            "max_batch", "max_ctx", "max_prefill_tokens", "model_kind",
                                            "local_hidden", "local_layers", "local_inter", "local_mlp_ffn",
                                            "eos_token_id")]


class MttsSampling(ctypes.Structure):
    _fields_ = [("text_temperature", ctypes.c_float), ("text_top_p", ctypes.c_float), ("text_top_k", ctypes.c_int),
                ("audio_temperature", ctypes.c_float), ("audio_top_p", ctypes.c_float), ("audio_top_k", ctypes.c_int),
                ("audio_repetition_penalty", ctypes.c_float), ("seed", ctypes.c_uint64)]


class MttsCodecStage(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("hidden", "layers", "n_heads", "n_kv", "head_dim", "inter", "upsample")]


MTTS_CODEC_MAX_STAGES = 8


class MttsCodecConfig(ctypes.Structure):
    _fields_ = [("n_q", ctypes.c_int), ("codebook_size", ctypes.c_int), ("n_stages", ctypes.c_int),
                ("stages", MttsCodecStage * MTTS_CODEC_MAX_STAGES), ("patch", ctypes.c_int),
                ("rope_theta", ctypes.c_float), ("rms_eps", ctypes.c_float),
                ("max_batch", ctypes.c_int), ("max_frames", ctypes.c_int), ("max_chunk_frames", ctypes.c_int)]


class MttsChannelSampling(ctypes.Structure):
    _fields_ = [("do_sample", ctypes.c_int), ("temperature", ctypes.c_float), ("top_k", ctypes.c_int),
                ("top_p", ctypes.c_float), ("repetition_penalty", ctypes.c_float)]


P = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float
SZ = ctypes.c_size_t
U64 = ctypes.c_uint64

# name -> (restype, argtypes)
_SIGS = {
    "mtts_last_error": (ctypes.c_char_p, []),
    "mtts_version": (I, []),
    "mtts_build_id": (ctypes.c_char_p, []),
    "mtts_engine_create": (I, [ctypes.POINTER(MttsConfig), I, ctypes.POINTER(P)]),
    "mtts_engine_destroy": (I, [P]),
    "mtts_engine_reserve": (I, [P, I, I, I]),
    "mtts_engine_load_weight": (I, [P, ctypes.c_char_p, P, SZ, I]),
    "mtts_engine_init_random": (I, [P, U64]),
    "mtts_engine_weight_bytes": (I, [P, ctypes.POINTER(U64)]),
    "mtts_engine_time_gemv": (I, [P, I, I, I, I, ctypes.POINTER(F), ctypes.POINTER(U64)]),
    "mtts_forward": (I, [P, P, P, I, I, I, P, P]),
    "mtts_heads_ld": (I, [P]),
    "mtts_pse_active": (I, [P]),
    "mtts_pse4_active": (I, [P]),
    "mtts_pse_long_active": (I, [P]),
    "mtts_local_lpse_active": (I, [P]),
    "mtts_pse_ctx_max": (I, [P]),
    "mtts_pse_inject_timeout": (I, [P]),
    "mtts_pse_check": (I, [P]),
    "mtts_engine_set_pse_lazy": (I, [P, I]),
    "mtts_engine_load_weight_stream": (I, [P, ctypes.c_char_p, P, SZ, I, P]),
    "mtts_engine_kv_write": (I, [P, I, I, I, I, P, P]),
    "mtts_engine_kv_fill": (I, [P, ctypes.c_uint16]),
    "mtts_pse_trace": (I, [P, ctypes.POINTER(U64), ctypes.c_size_t]),
    "mtts_generate_begin": (I, [P, P, P, I, I, I, ctypes.POINTER(MttsSampling), P, P]),
    "mtts_generate_decode": (I, [P, I, P]),
    "mtts_generate_stats": (I, [P, P]),
    "mtts_generate_poll": (I, [P, ctypes.POINTER(I), ctypes.POINTER(I), P]),
    "mtts_generate": (I, [P, P, P, I, I, I, ctypes.POINTER(MttsSampling), P, I, ctypes.POINTER(I), P]),
    "mtts_local_generate_begin": (I, [P, P, P, I, I, I, I, ctypes.POINTER(MttsSampling), P]),
    "mtts_local_generate_decode": (I, [P, I, P]),
    "mtts_local_set_sampling": (I, [P, ctypes.POINTER(MttsChannelSampling), I]),
    "mtts_local_generate": (I, [P, P, P, I, I, I, I, ctypes.POINTER(MttsSampling), I, ctypes.POINTER(I), P]),
    "mtts_local_forward": (I, [P, P, P, I, I, I, I, P, P, I, P]),
    "mtts_local_frame_bytes": (I, [P, I, ctypes.POINTER(U64)]),
    "mtts_k_moss_rmsnorm": (I, [P, P, P, I, I, F, P]),
    "mtts_k_local_pick": (I, [P, I, I, I, P, P, I, I, I, F, I, F, F, U64, I, P]),
    "mtts_generate_fetch": (I, [P, P, I, P]),
    "mtts_generate_logits": (I, [P, P, P]),
    "mtts_k_pack": (I, [P, P, I, I, I, I, I, P]),
    "mtts_k_packed_bytes": (SZ, [I, I]),
    "mtts_k_gemv": (I, [P, P, I, P, I, P, I, I, I, I, I, I, I, I, P]),
    "mtts_k_gemv_ex": (I, [P, P, I, P, I, P, I, I, I, I, I, P, I, I, P, F, P, I, I, P]),
    "mtts_k_gemm": (I, [P, P, I, P, I, P, I, I, I, I, I, P, I, P]),
    "mtts_k_gemm_packed": (I, [P, P, P, I, I, P, I, I, I, I, I, P, I, P, SZ, P]),
    "mtts_k_gemv_splitk_ws_bytes": (SZ, [I, I]),
    "mtts_k_gemv_splitk_splits": (I, [I, I, I]),
    "mtts_k_gemv_splitk": (I, [P, P, I, P, I, P, I, I, I, I, I, P, I, P, P]),
    "mtts_k_rmsnorm": (I, [P, SZ, SZ, P, P, I, I, F, P]),
    "mtts_k_embed": (I, [P, I, P, P, I, I, P, I, P]),
    "mtts_k_qk_norm_rope": (I, [P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, F, P]),
    "mtts_k_attention_ws_bytes": (SZ, [I, I, I, I]),
    "mtts_k_attention": (I, [P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, P]),
    "mtts_k_attention_prefill": (I, [P, P, P, P, P, P, I, I, I, I, I, I, P]),
    "mtts_k_attn_decode_ws_bytes": (SZ, [I, I, I, I, I]),
    "mtts_k_attn_decode": (I, [P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, P]),
    "mtts_rope_table": (I, [F, I, I, P, P]),
    "mtts_k_fill_uniform": (I, [P, SZ, U64, U64, F, F, P]),
    # codec decoder (include/mtts_codec.h)
    "mtts_codec_create": (I, [ctypes.POINTER(MttsCodecConfig), I, ctypes.POINTER(P)]),
    "mtts_codec_destroy": (I, [P]),
    "mtts_codec_load_weight": (I, [P, ctypes.c_char_p, P, SZ, I]),
    "mtts_codec_init_random": (I, [P, U64]),
    "mtts_codec_samples_per_frame": (I, [P]),
    "mtts_codec_position": (I, [P]),
    "mtts_codec_reset": (I, [P]),
    "mtts_codec_decode": (I, [P, P, I, I, I, I, P, SZ, P]),
    "mtts_codec_weight_bytes": (I, [P, ctypes.POINTER(U64)]),
}

EXPORTED = tuple(_SIGS)

_lib = None


def lib_path():
    return _LIB_PATH


def load():
    """Load libmtts.so (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise RuntimeError(f"libmtts.so not found at {_LIB_PATH}; build it with "
                           "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C moss_tts_amd/csrc`")
    lib = ctypes.CDLL(_LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if _LIB_PATH == _DEFAULT_LIB:
        # the in-tree library must have been built from this tree's sources (moss_tts_amd/_buildid.py)
        from . import _buildid
        built, tree = lib.mtts_build_id().decode(), _buildid.tree_hash("lib")
        if built != tree:
            raise RuntimeError(f"stale {_LIB_PATH}: built from sources {built[:16]}, the tree's are {tree[:16]}; "
                               "rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")
    _lib = lib
    return lib


def build_id():
    """the source hash compiled into the loaded libmtts.so"""
    return load().mtts_build_id().decode()


class PseTimeout(RuntimeError):
    """MTTS_E_PSE_TIMEOUT: a batch-1 persistent decode launch timed out; the logits of the
    forwards since the last check are invalid and the engine now runs the per-op launches."""


def check(rc, what=""):
    if rc == MTTS_OK:
        return
    msg = load().mtts_last_error().decode(errors="replace")
    if rc == MTTS_E_INVALID:
        raise ValueError(f"{what}: {msg}")
    if rc == MTTS_E_PSE_TIMEOUT:
        raise PseTimeout(f"{what} failed ({rc}): {msg}")
    raise RuntimeError(f"{what} failed ({rc}): {msg}")


def call(name, *args):
    rc = getattr(load(), name)(*args)
    check(rc, name)
    return rc
