/*
 * tic.h — C-ABI of libtic.so, the MI355X (gfx950) encode/decode hot path of the
 * learned image codec in bolin-chen/tf_image_compression.
 *
 * The reference has no FFI: its hot path is a TF-1.x graph built by
 * model_N.encoder/decoder and run by tf.Session.  Each entry point below names the
 * reference interface it replaces (paths relative to the reference root).  All
 * arguments are plain pointers and sizes; tensors are C-contiguous NHWC.  Every
 * function returns 0 on success or a negative TIC_E* code; tic_last_error()
 * returns a thread-local message for the last failure on the calling thread.
 *
 * Host pointers (tic_encode / tic_decode / tic_rmbe) are owned by the caller and are
 * only read/written during the call.  Device pointers (the *_device variants) must
 * come from tic_device_alloc on the same handle; those calls are asynchronous on the
 * handle's HIP stream — use tic_synchronize() before reading results.
 */
#ifndef TIC_H_
#define TIC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TIC_OK 0
#define TIC_EINVAL (-1)     /* bad argument / shape (reference: ValueError, tf.errors.InvalidArgumentError) */
#define TIC_ENOTFOUND (-2)  /* unknown variable name (reference: Saver.restore NotFoundError) */
#define TIC_ESTATE (-3)     /* handle not finalized / missing weights */
#define TIC_EHIP (-4)       /* HIP runtime error */
#define TIC_ENOMEM (-5)
#define TIC_EUNSUPPORTED (-6)
#define TIC_EOVERFLOW (-7)  /* value does not fit (reference: OverflowError) */
#define TIC_EIO (-8)        /* file I/O (reference: IOError / RuntimeError) */

#define TIC_MODEL_RMBE 100  /* submit/2/rmbe/model.py:113 (block-effect post-filter) */
#define TIC_MODEL_CH128 128 /* base_model/ch_128/model.py:34-215 (128-channel trunk, P/4 code) */

typedef struct tic_handle tic_handle;

/* Library / build identification. */
const char* tic_version(void);
const char* tic_last_error(void);

/* Open a codec for model_N on HIP device `device`.
 * Replaces: `from model_N import model` (encode.py:225-232, decode.py:280-287,
 *   submit/encoder.py:220-223) + model_N/config.json's patch_size/quan_scale
 *   (encode.py:129-145) + os.environ['CUDA_VISIBLE_DEVICES']=gpu (encode.py:218).
 * model_id: 0..3, TIC_MODEL_CH128 or TIC_MODEL_RMBE.  patch_size: even, >= 16 (for rmbe: 128).
 * quan_scale: Q in [2, 256] (model_0/config.json:6). */
int tic_create(int model_id, int patch_size, int quan_scale, int device, tic_handle** out);
void tic_destroy(tic_handle* h);

/* Channel statistics (float32 [3]).
 * Replaces: np.load('data_info/channel_normalization_params.npz') at model import
 *   (model_0/model.py:18,26-28; submit/2/rmbe/model.py:25-30). */
int tic_set_normalization(tic_handle* h, const float* mean3, const float* std3);

/* One TF variable, by its scope name and TF layout: '<scope>/kernel' HWIO [3,3,Cin,Cout]
 * for conv (basic_block/basic_block.py:30), [3,3,Cout,Cin] for conv-transpose (:53);
 * '<scope>/bias' [Cout] (:35,:59).  Copied and repacked at tic_finalize.
 * Replaces: tf.train.Saver().restore (utils/utils.py:84-93), one variable at a time. */
int tic_set_param(tic_handle* h, const char* name, const float* data, const int64_t* shape, int ndim);

/* Check every variable is present, repack and upload.  (Saver.restore's all-or-nothing.) */
int tic_finalize(tic_handle* h);

/* Shape of the quantised code for one patch (h, w, C).
 * Replaces: encoded_patches[0][0].shape (encode.py:171) / get_encoded_shape (decode.py:130-140). */
int tic_code_shape(const tic_handle* h, int* eh, int* ew, int* ec);

/* Encoder: uint8 RGB patches [n,P,P,3] -> uint8 symbols [n,eh,ew,ec] in {0..Q-1}
 * (optional float32 pre-quantiser activations [n,eh,ew,ec] for parity checks).
 * Replaces: model.encoder(input, patch_size, quan_scale) (model_0/model.py:34-144)
 *   + the sess.run loop (encode.py:157-165) + astype(int) (encode.py:182). */
int tic_encode(tic_handle* h, const uint8_t* patches, int n, uint8_t* idx_out, float* preact_out);

/* Decoder: uint8 symbols [n,eh,ew,ec] -> uint8 RGB [n,P,P,3] (np.around half-even of the
 * clipped float) and/or the float32 reconstruction in [0,255] (either may be NULL).
 * Replaces: model.decoder(input, quan_scale) (model_0/model.py:147-263) + sess.run loop
 *   (decode.py:212-220) + np.around(...).astype(np.uint8) (decode.py:249). */
int tic_decode(tic_handle* h, const uint8_t* idx, int n, uint8_t* rgb_out, float* f32_out);

/* Block-effect post-filter network on float32 RGB windows [n,128,128,3] -> float32 (clipped).
 * Handle must be created with TIC_MODEL_RMBE.
 * Replaces: rmbe_model.model(patch_batch) + sess.run (submit/2/rmbe/model.py:113-197,
 *   submit/2/rmbe/rmbe.py:28-67). */
int tic_rmbe(tic_handle* h, const float* windows, int n, float* out);

/* --- device-resident variants (benchmarks, multi-stage pipelines) --- */
int tic_device_alloc(tic_handle* h, size_t bytes, void** dptr);
int tic_device_free(tic_handle* h, void* dptr);
int tic_memcpy_h2d(tic_handle* h, void* dst, const void* src, size_t bytes);
int tic_memcpy_d2h(tic_handle* h, void* dst, const void* src, size_t bytes);
int tic_synchronize(tic_handle* h);
int tic_encode_device(tic_handle* h, const uint8_t* d_patches, int n, uint8_t* d_idx, float* d_preact);
int tic_decode_device(tic_handle* h, const uint8_t* d_idx, int n, uint8_t* d_rgb, float* d_f32);
/* encode then decode back-to-back on the handle's stream (the benchmark step). */
int tic_codec_device(tic_handle* h, const uint8_t* d_patches, int n, uint8_t* d_idx, uint8_t* d_rgb);
int tic_rmbe_device(tic_handle* h, const float* d_windows, int n, float* d_out);

/* Options: "streams" (1 or 2 execution lanes; with 2, every batch chunk is split in halves
 * on two HIP streams that run concurrently — default 2, env TIC_STREAMS), "chunk" (max
 * patches per launch sequence, default 256, env TIC_MAX_CHUNK), "graph" (1: replay
 * tic_codec_device as a captured HIP graph per (buffers, n) — default 0: measured slower
 * than eager dual-lane launches on MI355X), "persist_grid" (> 0: cap on the grid of the
 * persistent conv variants, so that tests run several tiles per workgroup; default 0).
 * Structural, bit-identical fusions (1 on, 0 off, -1 the model's default): "fuse01"
 * (encode_0 + encode_1 in one launch; default on), "fuse_tail" (decode_1 + decode_0; on),
 * "chain" (each run of stride-1 64->64 layers in one launch; on for models 0-2, off for
 * model_3 / rmbe; declined automatically where the geometry cannot run it), "chain_wh"
 * (1 or 2), "chain_x" (1: the encoder's stride-2 layer in front of a run and the decoder's
 * transposed layer behind it run inside the chain's launch; 2: also the decoder's next
 * transposed layer (decode_2); needs chain_wh 2; default 1 for models 0-2, the shipped tuning
 * decides), "chain_order" (region placement: 0 atomic ticket, 1 blockIdx, 2 a
 * patch's regions on one XCD, -1 automatic), "s1_form" (stride-1 form: 0 direct, 1 Winograd F(2x2,3x3), 2 Winograd F(4x4,3x3)
 * for the 64->64 res-block convs, other layers falling back to 1; -1 the model's default: 2 for
 * model_3 and the rmbe net, 1 otherwise; env TIC_S1_FORM=direct|wino|wino4), "s2_form" (standalone
 * stride-2 / transposed layers: 0 direct, 1 polyphase Winograd — layers a fused kernel could run
 * keep the direct form; -1 the model's default: 1 for models 0, 1 and 3 (80-channel layers direct), 0 otherwise; env TIC_S2_FORM=direct|pwino), "decouple" (lanes fork from the
 * handle stream only when a call's device byte ranges or earlier non-lane work require it;
 * default 1), "mark_layer" (see tic_mark_durations). */
int tic_set_option(tic_handle* h, const char* key, int value);

/* --- introspection / measurement --- */
int tic_num_layers(const tic_handle* h);
/* kind: 0 conv s1, 1 conv s2, 2 conv-transpose s2; act: 0 identity, 1 relu;
 * stage: 0 encoder, 1 decoder.  name_buf receives the TF scope (NUL-terminated). */
int tic_layer_info(const tic_handle* h, int i, char* name_buf, int name_len, int* kind, int* cin,
                   int* cout, int* act, int* stage, int* residual);
/* Static layer table keyed by model id (no handle, no device needed). */
int tic_model_num_layers(int model_id);
int tic_model_layer(int model_id, int i, char* name_buf, int name_len, int* kind, int* cin, int* cout,
                    int* act, int* stage, int* residual);
/* Time each layer's kernel with HIP events on the handle's stream over `iters` runs of
 * tic_codec_device(n) (or the rmbe net); writes the mean ms per launch of layer i to
 * ms_out[i] (size >= tic_num_layers). */
int tic_profile_layers(tic_handle* h, const void* d_in, int n, int iters, float* ms_out);
/* In-step launch timing (bench.py's roofline): with option "mark_layer" = i (>= 0) every
 * lane records a HIP event pair on its own stream around each launch that starts at layer i
 * (a fused or chained launch starts at its first layer) during ordinary tic_codec_device /
 * encode / decode calls, up to 1024 pairs per lane.  tic_mark_durations synchronises,
 * writes up to cap durations (ms) to ms_out, returns how many, and clears the record. */
int tic_mark_durations(tic_handle* h, float* ms_out, int cap);

/* Measure every compiled tiling of every layer on the live buffers of one encode+decode
 * (or rmbe) pass over d_in[n] and keep the fastest per layer for batch size n (like
 * cuDNN's benchmark mode).  Untuned batch sizes use a grid-size heuristic. */
int tic_autotune(tic_handle* h, const void* d_in, int n, int reps);
/* In-situ tuning for tic_codec_device / tic_rmbe_device on n patches: each layer's
 * variant is chosen by the time of the whole launch sequence as it runs (both lanes),
 * greedy over the layers for `rounds` passes, each candidate timed as `reps` steps (min
 * of 3).  Starts from tic_autotune's per-layer choice (run here if missing).  All
 * candidates produce bit-identical results. */
int tic_autotune_step(tic_handle* h, const void* d_in, int n, int rounds, int reps);
/* Tiling used by layer i for batch n: rows per workgroup and channel split, the latter
 * + 100 when the weights are staged through LDS (0,0 if the layer has one fixed kernel). */
int tic_layer_variant(const tic_handle* h, int i, int n, int* th, int* nsplit);
/* Kernel instance layer i launches for batch n, as "<kernel>" "<template args>" in the
 * form tools/pmc_summary.py prints (e.g. "conv3x3<1,32,32,4,4,1,false,1,false,0,0>");
 * empty when the layer runs inside the previous layer's launch.  cap includes the NUL. */
int tic_layer_kernel(const tic_handle* h, int i, int n, char* name, int cap);
/* Tuning state as text (every tuned tiling / variant per layer and batch key, and the
 * structural fusion flags), so a tuning run can be replayed exactly by another process of
 * the same build (like cuDNN's find-db): returns the length (excluding the NUL) and writes
 * it when cap is large enough.  tic_tuning_import validates every entry against the
 * layer table and the compiled registries (TIC_EINVAL on any mismatch, nothing applied). */
int tic_tuning_export(const tic_handle* h, char* buf, int cap);
int tic_tuning_import(tic_handle* h, const char* text);

/* Unit-test entry: one layer on device float32 NHWC tensors.
 * kind/act as tic_layer_info; res (nullable) is added after the activation.
 * w is the TF-layout kernel (HWIO for conv, [3,3,Cout,Cin] for conv-T), host memory.
 * in: [n,H,W,cin]; out: [n,Ho,Wo,cout]. */
int tic_conv3x3_device(tic_handle* h, int kind, int act, const float* d_in, int n, int H, int W, int cin,
                       int cout, const float* w_host, const float* b_host, const float* d_res, float* d_out);

/* The handle's HIP stream (hipStream_t as void*), e.g. to enqueue an RCCL collective
 * behind the codec's kernels.  Work enqueued there is ordered before every later codec
 * call: from this call on the handle's execution lanes fork from the stream at every call
 * (see tic_stream_external). */
int tic_get_stream(tic_handle* h, void** stream);
/* Declare whether the caller may have work of its own pending on the handle's stream
 * (1, the state after tic_get_stream) or synchronises everything it enqueues there before
 * the next codec call (0): then the lanes fork from the stream only after the handle's own
 * copies / glue kernels, and each lane starts its next batch as soon as it is free. */
int tic_stream_external(tic_handle* h, int on);

/* Device info string (name, CUs, arch) for logs. */
int tic_device_info(tic_handle* h, char* buf, int len);

/* --- whole images (BASELINE config 5) and symbol statistics; device pointers, async on
 * the handle's stream.  Any handle may run the glue kernels; tic_rmbe_image_device needs
 * a TIC_MODEL_RMBE handle. --- */

/* Reflect-pad an HWC uint8 image [H,W,3] bottom/right to multiples of P (np.pad 'reflect':
 * edge pixel not repeated, any pad length) and cut row-major PxP patches into
 * d_patches [ceil(H/P)*ceil(W/P), P, P, 3] (4-byte aligned; P a multiple of 4).
 * Replaces: utils.crop_image_input_patches (utils/utils.py:96-133), encode.py:154-156. */
int tic_image_to_patches_device(tic_handle* h, const uint8_t* d_img, int H, int W, int P, uint8_t* d_patches);

/* Stitch row-major float32 patches [ceil(H/P)*ceil(W/P), P, P, 3] into an HWC image cropped
 * to HxW.  Replaces: utils.concat_patches (utils/utils.py:136-167), decode.py:222-230. */
int tic_patches_to_image_device(tic_handle* h, const float* d_patches, int H, int W, int P, float* d_img);

/* Block-effect post-filter of a whole float32 HWC image [H,W,3] in [0,255], in place: the
 * 128x128 windows at column offset 64 (all full rows of windows), filtered and written back,
 * then the windows at row offset 64; edge strips that fill no window stay untouched.
 * Replaces: rmbe.rmbe / rmbe_height / rmbe_width (submit/2/rmbe/rmbe.py:15-111) with the
 * network of submit/2/rmbe/model.py:113-197 (one handle, no per-call graph rebuild). */
int tic_rmbe_image_device(tic_handle* h, float* d_img, int H, int W);

/* np.around(x).astype(np.uint8) of n float32 values in [0,255] (half to even; clamped).
 * Replaces: submit/2/decoder.py:176, decode.py:249. */
int tic_round_u8_device(tic_handle* h, const float* d_in, size_t n, uint8_t* d_out);

/* Accumulate np.histogram(symbols, bins=range(Q+1))[0] of n uint8 symbols into the uint64
 * counts d_counts[Q] (d_sym 4-byte aligned, d_counts 8-byte aligned; zero it first with
 * tic_memset_device).  Replaces: get_encoded_distribution.py:113-126 (the per-batch
 * histogram of the encoder output summed over the data set). */
int tic_histogram_device(tic_handle* h, const uint8_t* d_sym, size_t n, int Q, uint64_t* d_counts);

/* Accumulate the exact sum of squared differences of two uint8 arrays of n bytes into
 * *d_acc (uint64; 4-byte aligned inputs).  Replaces: evaluate.mse summed over a data set
 * (processing_utils/evaluate.py:10-32; dataset PSNR = 10 log10(255^2 sum(dims)/sum(SSE))). */
int tic_sse_u8_device(tic_handle* h, const uint8_t* d_a, const uint8_t* d_b, size_t n, uint64_t* d_acc);

/* hipMemsetAsync on the handle's stream. */
int tic_memset_device(tic_handle* h, void* d_ptr, int value, size_t bytes);

/* Make `waiter`'s stream wait for all work enqueued so far on `signaler`'s stream (same
 * device): chains a codec handle and an rmbe handle without a host synchronisation. */
int tic_stream_wait(tic_handle* waiter, tic_handle* signaler);
/* Named dependencies (slot 0..7): tic_event_record marks the point reached so far on h's
 * stream; tic_stream_wait_event makes `waiter`'s stream wait for the last mark of that
 * slot on `signaler` (no-op if never recorded).  Lets a pipeline wait for exactly the
 * work that last used a buffer (e.g. the rmbe pass of image i-2 before the codec of
 * image i reuses its stitch buffer) instead of everything enqueued so far. */
int tic_event_record(tic_handle* h, int slot);
int tic_stream_wait_event(tic_handle* waiter, tic_handle* signaler, int slot);

/* CRC-32C (Castagnoli) of n bytes, continuing `crc` (0 to start).  Host only.  Used by the
 * TensorFlow checkpoint reader that replaces tf.train.Saver.restore (utils/utils.py:84-93):
 * table blocks and tensor-bundle entries carry masked CRC-32C checksums. */
uint32_t tic_crc32c(const void* data, size_t n, uint32_t crc);

/* --- entropy coder (host, no device) ---
 * Replaces the third-party `range_coder` package used by encode.py:86-97 and
 * decode.py:89-99: RangeEncoder(path).encode(data, cum_freq) / .close() and
 * RangeDecoder(path).decode(n, cum_freq) / .close().  cum_freq: non-decreasing int64
 * table starting at 0, entries < 2^32 (else TIC_EOVERFLOW), total <= 2^24.  Symbols
 * with zero frequency or outside the table are TIC_EINVAL; calls after close are
 * TIC_ESTATE.  Several encode() calls append to one stream. */
typedef struct tic_rc_encoder tic_rc_encoder;
typedef struct tic_rc_decoder tic_rc_decoder;
const char* tic_rc_last_error(void);
int tic_rc_encoder_open(const char* path, tic_rc_encoder** out);
int tic_rc_encode(tic_rc_encoder* e, const int64_t* data, size_t n, const int64_t* cum_freq, size_t ncum);
int tic_rc_encoder_close(tic_rc_encoder* e);
void tic_rc_encoder_free(tic_rc_encoder* e);
int tic_rc_decoder_open(const char* path, tic_rc_decoder** out);
int tic_rc_decode(tic_rc_decoder* d, size_t n, const int64_t* cum_freq, size_t ncum, int64_t* out);
int tic_rc_decoder_close(tic_rc_decoder* d);
void tic_rc_decoder_free(tic_rc_decoder* d);

#ifdef __cplusplus
}
#endif

#endif /* TIC_H_ */
