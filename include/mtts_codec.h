/* mtts_codec.h -- C ABI of the codec decoder in libmtts.so (MOSS-Audio-Tokenizer decode side).
 *
 * Replaces the `processor.audio_tokenizer.decode(codes, padding_mask, return_dict=True,
 * chunk_duration=...)` seam of the reference processor (moss_tts_delay/processing_moss_tts.py:
 * 880-930, moss_tts_local/processing_moss_tts.py:913-923) and the streaming decode of
 * moss_tts_realtime (AudioStreamDecoder, streaming_mossttsrealtime.py:679-804).
 *
 * The codec's source and weights are not in the reference tree (the moss_audio_tokenizer
 * submodule is empty; README.md:382-393 describes it as "Cat": RVQ with 32 codebooks at
 * 12.5 Hz and a CNN-free stack of causal Transformer blocks).  The decoder built here follows
 * that description: residual-vector dequantisation (sum of the first n_q codebook rows, each
 * quantizer's output projection folded into its table), then stages of causal Transformer
 * blocks (Qwen3 block family: RMSNorm, GQA attention with q/k-norm and RoPE, SwiGLU), each
 * stage ending in an RMSNorm and a linear upsampling projection (dim -> upsample x next dim,
 * reshaped to upsample x the tokens), and a final linear projection of the last stage's tokens
 * to waveform patches.  Every shape is a config field; weights load by name.
 *
 * Decoding is causal and incremental: mtts_codec_decode continues from the frames already
 * decoded since the last mtts_codec_reset (KV caches per stage), so decoding a stream in
 * chunks gives the waveform of decoding it at once.  Errors and threading as in mtts.h.
 */
#ifndef MTTS_CODEC_H
#define MTTS_CODEC_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mtts_codec mtts_codec;

#define MTTS_CODEC_MAX_STAGES 8

typedef struct mtts_codec_stage {
  int hidden, layers, n_heads, n_kv, head_dim, inter;
  int upsample; /* tokens of the next stage per token of this one (1 for the last stage) */
} mtts_codec_stage;

typedef struct mtts_codec_config {
  int n_q;           /* codebooks (RVQ depth) */
  int codebook_size; /* rows per codebook */
  int n_stages;
  mtts_codec_stage stages[MTTS_CODEC_MAX_STAGES];
  int patch;         /* waveform samples per last-stage token */
  float rope_theta, rms_eps;
  /* capacity */
  int max_batch;        /* streams decoded together */
  int max_frames;       /* frames per stream between resets (KV capacity) */
  int max_chunk_frames; /* frames per forward (workspace); longer decodes are chunked */
} mtts_codec_config;

int mtts_codec_create(const mtts_codec_config* cfg, int device, mtts_codec** out);
int mtts_codec_destroy(mtts_codec* codec);
/* Weight names:
 *   quantizer.codebooks.{q}.weight                 [codebook_size, stages[0].hidden]
 *   decoder.stages.{s}.layers.{i}.<Qwen3 layer name>  (self_attn.{q,k,v,o}_proj.weight,
 *       self_attn.{q,k}_norm.weight, mlp.{gate,up,down}_proj.weight,
 *       input_layernorm.weight, post_attention_layernorm.weight)
 *   decoder.stages.{s}.norm.weight                 [hidden_s]
 *   decoder.stages.{s}.upsample.weight             [upsample_s * hidden_{s+1}, hidden_s]  (s < last)
 *   decoder.out_proj.weight                        [patch, hidden_last]
 * src: bf16 row-major, host (on_dev = 0) or device (1). */
int mtts_codec_load_weight(mtts_codec* codec, const char* name, const void* src, size_t bytes, int on_dev);
/* random weights (benchmarks), deterministic in seed */
int mtts_codec_init_random(mtts_codec* codec, uint64_t seed);
/* waveform samples per frame = patch x prod(upsample) */
int mtts_codec_samples_per_frame(const mtts_codec* codec);
/* frames decoded since the last reset */
int mtts_codec_position(const mtts_codec* codec);
/* start new streams: the next decode is frame 0 */
int mtts_codec_reset(mtts_codec* codec);
/* Decode T more frames of B streams.  codes_dev: int64 [B, T, ld_codes] (frame-major, the
 * first n_q_used entries of each frame are used: fewer codebooks = lower bitrate); wav_dev:
 * fp32 [B, ld_wav], ld_wav >= T * spf, receives the T frames' samples (stream samples
 * [pos * spf, (pos + T) * spf), pos = mtts_codec_position() before the call). */
int mtts_codec_decode(mtts_codec* codec, const int64_t* codes_dev, int B, int T, int ld_codes, int n_q_used,
                      float* wav_dev, size_t ld_wav, void* stream);
/* Weight bytes streamed per forward (roofline accounting). */
int mtts_codec_weight_bytes(const mtts_codec* codec, uint64_t* bytes);

#ifdef __cplusplus
}
#endif
#endif
