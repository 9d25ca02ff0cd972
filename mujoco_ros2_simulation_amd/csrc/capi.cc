// C ABI (include/mrs.h): exception firewall + handle management.  Every entry point catches, stores
// the message in a thread-local buffer (mrs_last_error) and returns an MRS_ERR_* code or NULL.
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

#include "../../include/mrs.h"
#include "hip/batch.h"
#include "mjcf/model.h"
#include "mjcf/xml.h"

struct mrs_model {
  mrs::Model m;
};
struct mrs_batch {
  mrs::BatchImpl* impl = nullptr;
  const mrs_model* model = nullptr;
};

namespace {

thread_local std::string g_last_error;
thread_local int g_last_code = MRS_OK;

void set_error(const std::string& msg) { g_last_error = msg; }

template <class F>
int guarded_impl(F&& f) {
  try {
    g_last_error.clear();
    f();
    return MRS_OK;
  } catch (const mrs::DeviceError& e) {
    set_error(e.what());
    return MRS_ERR_DEVICE;
  } catch (const mrs::UnsupportedError& e) {
    set_error(e.what());
    return MRS_ERR_UNSUPPORTED;
  } catch (const std::invalid_argument& e) {
    set_error(e.what());
    return MRS_ERR_INVALID;
  } catch (const std::exception& e) {
    set_error(e.what());
    return MRS_ERR_INVALID;
  } catch (...) {
    set_error("unknown error");
    return MRS_ERR_INVALID;
  }
}

template <class F>
int guarded(F&& f) {
  g_last_code = guarded_impl(f);
  return g_last_code;
}

bool ends_with(const std::string& s, const char* suffix) {
  const size_t n = std::strlen(suffix);
  return s.size() > n && s.compare(s.size() - n, n, suffix) == 0;
}

void copy_error(char* error, int error_len) {
  if (error && error_len > 0) {
    std::strncpy(error, g_last_error.c_str(), static_cast<size_t>(error_len) - 1);
    error[error_len - 1] = '\0';
  }
}

}  // namespace

extern "C" {

const char* mrs_last_error(void) { return g_last_error.c_str(); }
int mrs_last_status(void) { return g_last_code; }

mrs_model* mrs_model_load_xml(const char* path, char* error, int error_len) {
  std::unique_ptr<mrs_model> out;
  int rc = guarded([&] {
    if (!path || !*path) throw std::invalid_argument("empty model path");
    // the reference loads a path ending in ".mjb" with mj_loadModel (src/mujoco_system_interface.cpp:
    // 307-310): MuJoCo's binary format is a version-specific dump of mjModel that this compiler does
    // not read -- fail with MRS_ERR_UNSUPPORTED instead of handing binary data to the XML parser
    if (ends_with(path, ".mjb") || ends_with(path, ".MJB"))
      throw mrs::UnsupportedError(std::string("could not load binary model ") + path +
                                  ": MuJoCo .mjb files (mj_loadModel) are not supported, load the MJCF XML");
    out.reset(new mrs_model{mrs::compile_mjcf_file(path)});
  });
  if (rc != MRS_OK) {
    // parse / compile failures report MRS_ERR_LOAD; features outside the subset MRS_ERR_UNSUPPORTED
    if (rc != MRS_ERR_UNSUPPORTED) g_last_code = MRS_ERR_LOAD;
    copy_error(error, error_len);
    return nullptr;
  }
  if (error && error_len > 0) error[0] = '\0';
  return out.release();
}

mrs_model* mrs_model_load_xml_string(const char* xml, const char* basedir, char* error, int error_len) {
  std::unique_ptr<mrs_model> out;
  int rc = guarded([&] {
    if (!xml) throw std::invalid_argument("null XML string");
    out.reset(new mrs_model{mrs::compile_mjcf_string(xml, basedir ? basedir : ".")});
  });
  if (rc != MRS_OK) {
    // parse / compile failures report MRS_ERR_LOAD; features outside the subset MRS_ERR_UNSUPPORTED
    if (rc != MRS_ERR_UNSUPPORTED) g_last_code = MRS_ERR_LOAD;
    copy_error(error, error_len);
    return nullptr;
  }
  if (error && error_len > 0) error[0] = '\0';
  return out.release();
}

void mrs_model_free(mrs_model* m) { delete m; }

mrs_model* mrs_model_copy(const mrs_model* m) {
  std::unique_ptr<mrs_model> out;
  int rc = guarded([&] {
    if (!m) throw std::invalid_argument("null model");
    out.reset(new mrs_model{m->m});
  });
  return rc == MRS_OK ? out.release() : nullptr;
}

int mrs_model_view_get(const mrs_model* m, mrs_model_view* out) {
  return guarded([&] {
    if (!m || !out) throw std::invalid_argument("null argument");
    *out = m->m.view();
  });
}

int mrs_model_set_restate(mrs_model* m, int flags) {
  return guarded([&] {
    if (!m) throw std::invalid_argument("null model");
    if (flags & ~(MRS_RESTATE_NEWTON_REFINE | MRS_RESTATE_PGS_ELLIPTIC_BLOCK | MRS_RESTATE_NO_MPR_POLISH |
                  MRS_RESTATE_NO_MULTICCD))
      throw std::invalid_argument("unknown restate bits");
    m->m.restate = flags;
  });
}

int mrs_name2id(const mrs_model* m, int objtype, const char* name) {
  if (!m || !name) return -1;
  return m->m.name2id(objtype, name);
}

const char* mrs_id2name(const mrs_model* m, int objtype, int id) {
  if (!m) return nullptr;
  return m->m.id2name(objtype, id);
}

// getActuatorType (src/mujoco_system_interface.cpp:433-460): MOTOR if no bias; POSITION if affine
// bias with biasprm[1] != 0; VELOCITY if affine with biasprm[1] == 0 and biasprm[2] != 0; else CUSTOM
int mrs_actuator_type(const mrs_model* m, int id) {
  if (!m || id < 0 || id >= m->m.nu) return 0;
  const mrs::Model& mm = m->m;
  const int biastype = mm.actuator_biastype[id];
  const double* bp = &mm.actuator_biasprm[static_cast<size_t>(id) * MRS_NBIAS];
  if (biastype == MRS_BIAS_NONE) return 1;
  if (biastype == MRS_BIAS_AFFINE && bp[1] != 0) return 2;
  if (biastype == MRS_BIAS_AFFINE && bp[1] == 0 && bp[2] != 0) return 3;
  return 4;
}

mrs_batch* mrs_batch_create(const mrs_model* m, int n_envs, int device) {
  std::unique_ptr<mrs_batch> b(new mrs_batch());
  int rc = guarded([&] {
    if (!m) throw std::invalid_argument("null model");
    b->model = m;
    b->impl = mrs::batch_create(&m->m, n_envs, device, 0);  // contact capacity from the model
  });
  return rc == MRS_OK ? b.release() : nullptr;
}

void mrs_batch_free(mrs_batch* b) {
  if (!b) return;
  guarded([&] { mrs::batch_free(b->impl); });
  delete b;
}

int mrs_batch_num_envs(const mrs_batch* b) { return b ? mrs::batch_num_envs(b->impl) : 0; }

int mrs_batch_set_stream(mrs_batch* b, void* stream) {
  return guarded([&] {
    if (!b) throw std::invalid_argument("null batch");
    mrs::batch_set_stream(b->impl, stream);
  });
}

int mrs_batch_reset(mrs_batch* b, int key, int env0, int n) {
  return guarded([&] {
    if (!b) throw std::invalid_argument("null batch");
    mrs::batch_reset(b->impl, key, env0, n);
  });
}

int mrs_batch_set_field(mrs_batch* b, int field, const double* host, int env0, int n) {
  return guarded([&] {
    if (!b || !host) throw std::invalid_argument("null argument");
    mrs::batch_set(b->impl, field, host, env0, n);
  });
}

int mrs_batch_get_field(mrs_batch* b, int field, double* host, int env0, int n) {
  return guarded([&] {
    if (!b || !host) throw std::invalid_argument("null argument");
    mrs::batch_get(b->impl, field, host, env0, n);
  });
}

void* mrs_batch_device_ptr(mrs_batch* b, int field) {
  if (!b || field < 0 || field >= MRS_FIELD_COUNT) return nullptr;
  return mrs::batch_device_ptr(b->impl, field);
}

int mrs_batch_set_ctrl_device(mrs_batch* b, const float* d_ctrl) {
  return guarded([&] {
    if (!b || !d_ctrl) throw std::invalid_argument("null argument");
    mrs::batch_set_ctrl_device(b->impl, d_ctrl);
  });
}

int mrs_batch_bind_ctrl_device(mrs_batch* b, const float* d_ctrl) {
  return guarded([&] {
    if (!b) throw std::invalid_argument("null batch");
    mrs::batch_bind_ctrl_device(b->impl, d_ctrl);
  });
}

int mrs_batch_step(mrs_batch* b, int n_steps) {
  return guarded([&] {
    if (!b) throw std::invalid_argument("null batch");
    mrs::batch_launch(b->impl, n_steps, false);
  });
}

int mrs_batch_forward(mrs_batch* b) {
  return guarded([&] {
    if (!b) throw std::invalid_argument("null batch");
    mrs::batch_launch(b->impl, 1, true);
  });
}

int mrs_batch_render_depth(mrs_batch* b, int cam, int env0, int n, float* host_out) {
  return guarded([&] {
    if (!b || !host_out) throw std::invalid_argument("null argument");
    mrs::batch_render_depth(b->impl, cam, env0, n, host_out, false);
  });
}

int mrs_batch_render_depth_device(mrs_batch* b, int cam, int env0, int n, float* d_out) {
  return guarded([&] {
    if (!b || !d_out) throw std::invalid_argument("null argument");
    mrs::batch_render_depth(b->impl, cam, env0, n, d_out, true);
  });
}

int mrs_batch_render_rgbd(mrs_batch* b, int cam, int env0, int n, float* host_depth, unsigned char* host_rgb) {
  return guarded([&] {
    if (!b || !host_depth || !host_rgb) throw std::invalid_argument("null argument");
    mrs::batch_render_depth(b->impl, cam, env0, n, host_depth, false, host_rgb);
  });
}

int mrs_batch_render_rgbd_device(mrs_batch* b, int cam, int env0, int n, float* d_depth, unsigned char* d_rgb) {
  return guarded([&] {
    if (!b || !d_depth || !d_rgb) throw std::invalid_argument("null argument");
    mrs::batch_render_depth(b->impl, cam, env0, n, d_depth, true, d_rgb);
  });
}

int mrs_batch_render_async(mrs_batch* b, int cam, int env0, int n, float* d_depth, unsigned char* d_rgb) {
  return guarded([&] {
    if (!b || !d_depth) throw std::invalid_argument("null argument");
    mrs::batch_render_async(b->impl, cam, env0, n, d_depth, d_rgb);
  });
}

int mrs_batch_render_wait(mrs_batch* b) {
  return guarded([&] {
    if (!b) throw std::invalid_argument("null batch");
    mrs::batch_render_wait(b->impl);
  });
}

int mrs_batch_get_contacts(mrs_batch* b, int env, int max, int* geom, double* dist, double* pos, double* frame) {
  int ncon = 0;
  const int rc = guarded([&] {
    if (!b) throw std::invalid_argument("null batch");
    ncon = mrs::batch_get_contacts(b->impl, env, max, geom, dist, pos, frame);
  });
  return rc == MRS_OK ? ncon : rc;
}

int mrs_batch_get_efc(mrs_batch* b, int env, int max, int* type, double* J, double* R, double* aref,
                      double* force) {
  int nefc = 0;
  const int rc = guarded([&] {
    if (!b) throw std::invalid_argument("null batch");
    nefc = mrs::batch_get_efc(b->impl, env, max, type, J, R, aref, force);
  });
  return rc == MRS_OK ? nefc : rc;
}

int mrs_batch_get_field_device(mrs_batch* b, int field, float* d_out, int env0, int n) {
  return guarded([&] {
    if (!b || !d_out) throw std::invalid_argument("null argument");
    mrs::batch_get_field_device(b->impl, field, d_out, env0, n);
  });
}

int mrs_batch_sync(mrs_batch* b) {
  return guarded([&] {
    if (!b) throw std::invalid_argument("null batch");
    mrs::batch_sync(b->impl);
  });
}

int mrs_batch_set_timing(mrs_batch* b, int mask) {
  return guarded([&] {
    if (!b || mask < 0 || mask > 3) throw std::invalid_argument("timing mask must be 0..3");
    mrs::batch_set_timing(b->impl, mask);
  });
}

double mrs_batch_last_kernel_ms(mrs_batch* b, int kind) {
  double ms = -1;
  guarded([&] {
    if (!b) throw std::invalid_argument("null batch");
    ms = mrs::batch_last_kernel_ms(b->impl, kind);
  });
  return ms;
}

int mrs_debug_phase_cycles(double* out, int n, int reset) {
  if (!out || n < 0) return MRS_ERR_INVALID;
  return mrs::phase_cycles(out, n, reset != 0);
}

int mrs_debug_batch_layout(const mrs_batch* b, int* out, int n) {
  if (!b || !out || n < 0) return MRS_ERR_INVALID;
  return mrs::batch_layout(b->impl, out, n);
}

}  // extern "C"
