// Host-side sanitizer driver (test infrastructure, built by tests/test_sanitizers.py with
// -fsanitize=address,undefined): the MJCF compiler (product host code) on every benchmark and
// reference scene plus malformed inputs, and the fp64 oracle stepping each compiled model.  GPU code
// cannot run under AddressSanitizer on this pool, so the host paths are checked here.
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../mujoco_ros2_simulation_amd/csrc/mjcf/model.h"
extern "C" {
#include "../../oracle/oracle.h"
}

int main(int argc, char** argv) {
  int failures = 0;
  for (int i = 1; i < argc; ++i) {
    const std::string path = argv[i];
    try {
      mrs::Model model = mrs::compile_mjcf_file(path);
      mrs_model_view v = model.view();
      orc_data* d = orc_make_data(&v);
      orc_reset(&v, d, -1);
      for (int s = 0; s < 50; ++s) orc_step(&v, d);
      orc_forward(&v, d);
      if (v.ncam > 0) {
        std::vector<float> depth(static_cast<size_t>(v.cam_resolution[0]) * v.cam_resolution[1]);
        orc_render_depth(&v, d, 0, depth.data());
      }
      orc_free_data(d);
      std::printf("ok %s\n", path.c_str());
    } catch (const std::exception& e) {
      std::printf("FAIL %s: %s\n", path.c_str(), e.what());
      ++failures;
    }
  }
  // malformed or unsupported inputs must be rejected with an exception, never read out of bounds
  const char* bad[] = {
      "", "<mujoco", "<mujoco><worldbody><body><geom type=\"box\"/></body></worldbody>",
      "<mujoco><worldbody><geom type=\"mesh\"/></worldbody></mujoco>",
      "<mujoco><worldbody><body><joint type=\"hinge\" range=\"1\"/><geom size=\"0.1\"/></body></worldbody></mujoco>",
      "<mujoco><option cone=\"elliptic\"/><worldbody/></mujoco>",
      "<mujoco><worldbody><geom type=\"sphere\" size=\"-1 x\"/></worldbody></mujoco>",
      "<mujoco><worldbody><replicate count=\"-3\"><site/></replicate></worldbody></mujoco>",
      "<mujoco><asset><mesh name=\"m\" vertex=\"0 0 0 1 0\"/></asset><worldbody><geom type=\"mesh\" mesh=\"m\"/></worldbody></mujoco>",
  };
  // an empty model (every integrator) must step without touching absent arrays
  for (const char* integ : {"Euler", "RK4", "implicit", "implicitfast"}) {
    try {
      mrs::Model model = mrs::compile_mjcf_string(std::string("<mujoco><option integrator=\"") + integ +
                                                      "\"/><worldbody/></mujoco>", ".");
      mrs_model_view v = model.view();
      orc_data* d = orc_make_data(&v);
      orc_reset(&v, d, -1);
      orc_step(&v, d);
      orc_free_data(d);
    } catch (const std::exception& e) {
      std::printf("FAIL empty model (%s): %s\n", integ, e.what());
      ++failures;
    }
  }
  int rejected = 0;
  for (const char* xml : bad) {
    try {
      mrs::Model model = mrs::compile_mjcf_string(xml, ".");
      mrs_model_view v = model.view();
      orc_data* d = orc_make_data(&v);
      orc_reset(&v, d, -1);
      orc_step(&v, d);
      orc_free_data(d);
    } catch (const std::exception&) {
      ++rejected;
    }
  }
  std::printf("rejected %d of %zu malformed inputs\n", rejected, sizeof(bad) / sizeof(bad[0]));
  return failures ? 1 : 0;
}
