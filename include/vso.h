/*
 * vso.h — ONNX model sessions on gfx950: the part of onnxruntime-web the
 * reference uses to run its models, behind the same kind of C ABI as
 * ORT-web's own wasm exports (client/public/ort-wasm-simd-threaded.mjs:50-53).
 *
 * The reference creates ORT sessions for MODNet (initializeModnet,
 * client/src/core/model.ts:12-29; the weights file model_q4f16.onnx is absent
 * here), the MediaPipe face detector (initializeFaceDetector, model.ts:36-53,
 * client/src/assets/MediaPipeFaceDetector.onnx) and the landmark model
 * (initializeLandmarks, model.ts:58-67), and calls session.run on them
 * (frameProcessorTest.ts:91, :406, :478).  A vso_session parses an ONNX
 * ModelProto with its own protobuf reader, infers every shape for the
 * session's input shape, folds the shape arithmetic, and runs the graph as a
 * fixed list of HIP kernels (dense convolutions as implicit GEMMs on MFMA —
 * f32, or bf16 / f16 operands by option — depthwise convolutions direct, activations and
 * residual adds fused into the convolution epilogues), replayed from a
 * hipGraph.  Tensors are float32 NCHW.
 *
 * Supported operators: Conv, Relu, PRelu, LeakyRelu, Clip, Sigmoid, Tanh,
 * Add, Sub, Mul, Div (numpy broadcasting), MaxPool, AveragePool,
 * GlobalAveragePool, Pad (constant), Concat, Split, Slice, Transpose,
 * Reshape, Flatten, Squeeze, Unsqueeze, Identity, Dropout, Cast (float),
 * Resize/Upsample (nearest, linear; half_pixel, pytorch_half_pixel,
 * align_corners, asymmetric), InstanceNormalization, BatchNormalization,
 * MatMul, Gemm, Softmax, and Shape, Gather, Constant, ConstantOfShape,
 * Floor, Ceil, Cast on constants.  For q4f16 exports (model_q4f16.onnx's
 * form): float16 initializers, Cast to FLOAT16 (values rounded to halves and
 * kept as f32; later ops compute in f32), DequantizeLinear of int8 / uint8 /
 * int4 / uint4 weights (per tensor, per axis, opset-21 blocks; folded at
 * create) and com.microsoft MatMulNBits (4-bit blocks, packed uint8 zero
 * points, bias; dequantised once at create).  Anything else fails vso_create
 * with VSO_E_UNSUPPORTED naming the node.
 *
 * Errors: int returns are 0 or a negative code, message in vso_last_error
 * (thread-local when the session is NULL), like _OrtGetLastError (:50).
 * One call in flight per session.
 */
#ifndef VSO_H_
#define VSO_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  VSO_OK = 0,
  VSO_E_INVALID_ARG = -1,
  VSO_E_HIP = -2,
  VSO_E_PARSE = -3,
  VSO_E_UNSUPPORTED = -4,
  VSO_E_OOM = -5
};

typedef struct vso_session vso_session;

/* Session options (the part of ORT's SessionOptions this runtime has).
 * conv_precision: operands of the dense k x k convolutions (k_conv_tile,
 * vso_conv.hip) — VSO_PRECISION_F32: exact f32 products
 * (v_mfma_f32_16x16x4_f32), the default; _BF16 / _F16: activations and weights
 * rounded to bfloat16 / float16 (nearest even) on
 * v_mfma_f32_16x16x32_{bf16,f16}, f32 accumulation.  _F16 keeps every
 * float16-typed weight of a q4f16 export exact. */
enum { VSO_PRECISION_F32 = 0, VSO_PRECISION_BF16 = 1, VSO_PRECISION_F16 = 2 };
typedef struct vso_options {
  int conv_precision;
  int reserved[7];
} vso_options;

void vso_options_default(vso_options* o);

/* Replaces InferenceSession.create(url) (model.ts:14) / _OrtCreateSession(modelPtr,
 * len, opts) (ort-wasm-simd-threaded.mjs:51): model = the ONNX file's bytes.
 * input_dims/input_ndim: the shape of input 0 when the model leaves dims
 * symbolic (NULL/0 = the model's own static shape).  device_id: HIP ordinal. */
int vso_create(const void* model, size_t bytes, const int64_t* input_dims, int input_ndim, int device_id,
               vso_session** out);

/* vso_create with options (NULL = vso_options_default): InferenceSession.create(url, options). */
int vso_create_ex(const void* model, size_t bytes, const int64_t* input_dims, int input_ndim, int device_id,
                  const vso_options* opts, vso_session** out);

/* Replaces InferenceSession.release / _OrtReleaseSession (:51). */
void vso_destroy(vso_session* s);

/* Replaces _OrtGetLastError (:50). */
const char* vso_last_error(const vso_session* s);

/* Replaces _OrtGetInputOutputCount (:51). */
int vso_io_count(const vso_session* s, int* n_inputs, int* n_outputs);

/* Names (session.inputNames / outputNames) and shapes of inputs / outputs:
 * return the string length / the rank, or a negative code. */
int vso_input_name(const vso_session* s, int i, char* buf, int cap);
int vso_output_name(const vso_session* s, int i, char* buf, int cap);
int vso_input_shape(const vso_session* s, int i, int64_t* dims, int cap);
int vso_output_shape(const vso_session* s, int i, int64_t* dims, int cap);

/* Replaces session.run(feeds) (frameProcessorTest.ts:91) / _OrtRun (:53) for
 * host buffers: inputs[i] = float32 data of input i (its shape as above),
 * outputs[i] = room for output i.  Synchronous. */
int vso_run(vso_session* s, const float* const* inputs, float* const* outputs);

/* Device-resident variant: HBM pointers, enqueued on `stream` (hipStream_t;
 * NULL = the session's stream), not waited for. */
int vso_run_device(vso_session* s, const float* const* d_inputs, float* const* d_outputs, void* stream);

/* Introspection: the number of kernel launches per run, and launch k's
 * kernel name as rocprofv3 reports it (returns the string length). */
int vso_launch_count(const vso_session* s);
int vso_launch_name(const vso_session* s, int k, char* buf, int cap);
/* Convolutions planned on the LDS-tiled MFMA kernel (k_conv_tile). */
int vso_tile_conv_count(const vso_session* s);
/* Inverted residual blocks (1x1 expand -> Clip -> 3x3 depthwise -> Clip -> 1x1
 * project [-> + input]) the session runs as one fused launch each (MODNet's
 * MobileNetV2 backbone): k_ir in f32 sessions, k_ir_b16 (bf16 hi / lo splits
 * of both 1x1 operands, ~f32 precision) in bf16 / f16 ones, plus a
 * k_ir_reduce launch when the hidden channels are split over workgroups.
 * Planning knobs, read once per process: VSO_IR=0 plans them as three
 * launches; VSO_IR_B16=0 keeps the f32 form in 16-bit sessions; VSO_IR_CPS
 * (default 6) hidden 16-channel chunks per slice of a 16-bit block. */
int vso_ir_block_count(const vso_session* s);
/* Lanes of the captured graph (0 before the first run): launches that share no
 * activation buffer run on two capture streams, so independent branches of
 * the model (MODNet's HR branch beside its backbone) execute concurrently —
 * for sessions whose input 0 holds >= 2^21 elements; smaller ones capture one
 * stream (the cross-lane event edges cost more than the overlap there).
 * VSO_LANES=1 / 2 (read once per process) forces either. */
int vso_lane_count(const vso_session* s);

#ifdef __cplusplus
}
#endif

#endif /* VSO_H_ */
