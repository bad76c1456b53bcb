/*
 * ggml-q2a.h — the MI355X (gfx950) ggml backend of this repository: lib/libggml-q2a.so.
 *
 * A ggml backend plugin in the shape of the reference's own GPU backends (ggml/include/ggml-cuda.h:22-44): the
 * reference's whisper_full() builds its conv and encoder graphs unchanged (src/qwen2-whisper.cpp:1892-2203),
 * ggml_backend_sched splits them by supports_op, and graph_compute runs every node of the hot path on the GPU with
 * this repository's HIP kernels — including the nodes no shipped backend accepts, MUL_MAT(F32 im2col, F16 conv
 * kernel) and POOL_1D, so F16 / Q4_K / Q8_0 / Q4_0 model files run without the CPU split.
 *
 * Vtables implemented (ggml/src/ggml-backend-impl.h): ggml_backend_buffer_type_i :15-27, ggml_backend_buffer_i
 * :39-57, ggml_backend_i :86-133, ggml_backend_device_i :153-196, ggml_backend_reg_i :208-218.
 *
 * The plugin is compiled against ggml's headers (GGML_DIR in the package Makefile) and resolves ggml's own
 * functions (ggml_nbytes, ggml_backend_buffer_init, ...) from the application's ggml at load time, like a backend
 * built into libggml. Integration into whisper.cpp: INTEGRATION.md §"ggml backend".
 */
#pragma once

#include "ggml.h"
#include "ggml-backend.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GGML_Q2A_NAME "Q2A"
#define GGML_Q2A_MAX_DEVICES 16

/* backend (one HIP stream) on HIP device `device`; NULL if the device does not exist */
GGML_API ggml_backend_t ggml_backend_q2a_init(int device);          /* replaces ggml_backend_cuda_init, ggml-cuda.h:23 */
GGML_API bool ggml_backend_is_q2a(ggml_backend_t backend);          /* ggml_backend_is_cuda, ggml-cuda.h:25 */

/* device memory buffer type (weights and compute buffers) */
GGML_API ggml_backend_buffer_type_t ggml_backend_q2a_buffer_type(int device);   /* ggml-cuda.h:28 */

/* pinned (page-locked, portable) host buffer type for the CPU-side buffers whose bytes cross PCIe (inputs staged by
 * the CPU backend, results read back); replaces ggml_backend_cuda_host_buffer_type, ggml-cuda.h:34. Behaves as a CPU
 * buffer (is_host); GGML_Q2A_NO_PINNED=1 or a failed pinning gives a plain CPU buffer. Also the device's
 * get_host_buffer_type (ggml_backend_dev_host_buffer_type) */
GGML_API ggml_backend_buffer_type_t ggml_backend_q2a_host_buffer_type(void);

/* page-lock / release memory the caller owns; opt-in through GGML_Q2A_REGISTER_HOST (the reference's
 * GGML_CUDA_REGISTER_HOST): false when not enabled or refused. Replace ggml_backend_cuda_register_host_buffer /
 * _unregister_host_buffer, ggml-cuda.h:40-41; also reachable as "ggml_backend_register_host_buffer" /
 * "ggml_backend_unregister_host_buffer" through ggml_backend_reg_get_proc_address(ggml_backend_q2a_reg(), name).
 * (ggml_backend_cuda_split_buffer_type, ggml-cuda.h:31, has no counterpart: models are replicated per device.) */
GGML_API bool ggml_backend_q2a_register_host_buffer(void * buffer, size_t size);
GGML_API void ggml_backend_q2a_unregister_host_buffer(void * buffer);

GGML_API int  ggml_backend_q2a_get_device_count(void);                                           /* ggml-cuda.h:36 */
GGML_API void ggml_backend_q2a_get_device_description(int device, char * description, size_t description_size);
GGML_API void ggml_backend_q2a_get_device_memory(int device, size_t * free, size_t * total);      /* ggml-cuda.h:38 */

GGML_API ggml_backend_reg_t ggml_backend_q2a_reg(void);             /* ggml-cuda.h:43 */

/* statistics of the last graph_compute on this backend (test / profiling aid): kernels launched per node kind; nodes
 * folded into their producer's kernel (MUL_MAT -> ADD bias [-> GELU | ADD residual], NORM -> MUL -> ADD;
 * GGML_Q2A_NO_FUSE=1 disables it); whether the launches were replayed from a captured HIP graph (a cgraph seen
 * before; GGML_Q2A_NO_GRAPH=1 disables it) */
typedef struct {
    int n_nodes, n_mul_mat_fast, n_mul_mat_f32, n_attn_fused, n_other;
    int n_graph_replayed;
    int n_fused;
    int n_mm_grouped;   /* launches that ran several weight MUL_MATs of the same activation together: a layer's Q, K,
                           V projections as one GEMM writing the fused attention's operands (GGML_Q2A_NO_FUSED_QKV=1
                           disables it: then K|Q as one launch and V), or K|Q alone */
    int n_mul_mat_conv; /* MUL_MAT(F32 im2col, F16 kernel) on the fp16 MFMA GEMM with hi/lo-split activations */
    int n_buffer_reallocs; /* backend lifetime: scratch / V^T / fp16-shadow reallocations (each drops every captured
                              HIP graph, whose launches hold those buffers' addresses) */
    int n_mul_mat_conv_total; /* backend lifetime: n_mul_mat_conv summed over every graph_compute that ran its nodes */
    int n_repack_lazy;  /* backend lifetime: weights repacked at their first MUL_MAT (a device->host copy + host pack)
                           because their upload was not a whole host write the buffer could pack on arrival */
} ggml_backend_q2a_stats;
GGML_API void ggml_backend_q2a_get_stats(ggml_backend_t backend, ggml_backend_q2a_stats * stats);

#ifdef __cplusplus
}
#endif
