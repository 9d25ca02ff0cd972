// Internal C++ interface between the C ABI (capi.cc) and the HIP batch implementation.
#pragma once

#include <stdexcept>
#include <string>

namespace mrs {

struct Model;
struct BatchImpl;

struct DeviceError : std::runtime_error { using std::runtime_error::runtime_error; };
struct UnsupportedError : std::runtime_error { using std::runtime_error::runtime_error; };

BatchImpl* batch_create(const Model* model, int n_envs, int device, int max_contacts);
void batch_free(BatchImpl* b);
int batch_num_envs(const BatchImpl* b);
int batch_layout(const BatchImpl* b, int* out, int n);  // diagnostics: kernel configuration
void batch_set_stream(BatchImpl* b, void* stream);
void batch_reset(BatchImpl* b, int key, int env0, int n);
void batch_set(BatchImpl* b, int field, const double* host, int env0, int n);
void batch_get(BatchImpl* b, int field, double* host, int env0, int n);
void* batch_device_ptr(BatchImpl* b, int field);
void batch_set_ctrl_device(BatchImpl* b, const float* d_ctrl);
void batch_bind_ctrl_device(BatchImpl* b, const float* d_ctrl);  // zero-copy ctrl source (null: own buffer)
void batch_set_timing(BatchImpl* b, int mask);  // launches timed for batch_last_kernel_ms (bit 0 step, 1 frames)
void batch_launch(BatchImpl* b, int n_steps, bool forward_only);
// rgb (may be null): n * H * W * 3 bytes, same host/device side as out
void batch_render_depth(BatchImpl* b, int cam, int env0, int n, float* out, bool device_out, unsigned char* rgb = nullptr);
void batch_render_async(BatchImpl* b, int cam, int env0, int n, float* d_out, unsigned char* d_rgb);
void batch_render_wait(BatchImpl* b);
int batch_get_contacts(BatchImpl* b, int env, int max, int* geom, double* dist, double* pos, double* frame);
int batch_get_efc(BatchImpl* b, int env, int max, int* type, double* J, double* R, double* aref, double* force);
void batch_get_field_device(BatchImpl* b, int field, float* d_out, int env0, int n);
void batch_sync(BatchImpl* b);
double batch_last_kernel_ms(BatchImpl* b, int kind);
int phase_cycles(double* out, int n, bool reset);  // step.hip; profiling builds only

}  // namespace mrs
