// mjModel / mjData as the plugin keeps and exchanges them: the types of the reference's
// get_model(mjModel*&) / get_data(mjData*&) / set_data(mjData*)
// (include/mujoco_ros2_control/mujoco_system_interface.hpp:77-100, src/mujoco_system_interface.cpp:
// 1794-1814) and of its "mj_data_" / "mj_data_control_" double buffer (:684-688, 1756-1762).
//
// MuJoCo is not linked.  mjModel is the compiled model's flat view (include/mrs_model.h, field names
// are mjModel's: m->nq, m->jnt_qposadr[j], m->sensor_adr[s], ...) plus mjOption under m->opt; it
// owns a private copy of the compiled model, so a copy outlives the plugin exactly as
// mj_copyModel's does.  mjData holds the host mirror of one environment's state arrays under
// mjData's names, in one allocation.  The five lifecycle functions keep MuJoCo's names and
// argument conventions (dest == nullptr allocates); they are this library's own.
#pragma once

#include "mrs.h"
#include "mrs_model.h"

struct mjOption_ {
  double timestep;
  double gravity[3];
  double tolerance, impratio, ls_tolerance;
  int integrator, solver, iterations, ls_iterations, cone, disableflags;
};
typedef struct mjOption_ mjOption;

struct mjModel_ : mrs_model_view {
  mjOption opt;
  mrs_model* handle;  // compiled model this mjModel owns (mj_deleteModel frees it)
};
typedef struct mjModel_ mjModel;

struct mjData_ {
  double time;
  double* qpos;            // nq
  double* qvel;            // nv
  double* qacc;            // nv
  double* qacc_warmstart;  // nv
  double* ctrl;            // nu
  double* qfrc_applied;    // nv
  double* qfrc_actuator;   // nv
  double* sensordata;      // nsensordata
  int nq, nv, nu, nsensordata;  // sizes the arrays were made for (mj_copyData checks them)
  double* buffer;               // the one allocation behind the arrays
};
typedef struct mjData_ mjData;

// mjModel over a compiled model; takes ownership of `handle` (nullptr on a null handle)
mjModel* mj_wrapModel(mrs_model* handle);
// deep copy of src into dest (dest == nullptr: a new mjModel); returns dest
mjModel* mj_copyModel(mjModel* dest, const mjModel* src);
void mj_deleteModel(mjModel* m);
// zero-initialised mjData sized for m
mjData* mj_makeData(const mjModel* m);
// copy every array and the time of src into dest (dest == nullptr: a new mjData); returns dest,
// nullptr if dest and src were made for different sizes
mjData* mj_copyData(mjData* dest, const mjModel* m, const mjData* src);
void mj_deleteData(mjData* d);
