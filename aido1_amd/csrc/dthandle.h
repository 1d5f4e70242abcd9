// Internal: the opaque dt_handle behind include/dtsim.h, shared by the step
// (dtsim.hip) and observation (dtrender.hip) translation units.
#pragma once
#include <string>

#include "dtrender.h"
#include "dtsim_common.h"

struct StepCfg {
  int32_t repeat, frame_skip, action_mode, clip, speed_measured, auto_reset;
  uint32_t max_steps, max_env_steps, max_spawn_attempts;
  double reward_scale;
};

struct dt_handle {
  int device = 0;
  int n = 0;
  dt_config cfg{};
  dt::Geo geo{};
  StepCfg sc{};
  dt::MapDev map{};
  void* map_buf = nullptr;
  dt::State st{};
  void* st_buf = nullptr;
  size_t lds_bytes = 0;
  uint32_t env_base = 0;
  // observation path (dtrender.hip)
  dt_line_params line_params{};
  dr::LineDev line{};
  void* mark_buf = nullptr;   // float4 segments (x0, z0, x1, z1): yellow then white
  int32_t n_yellow = 0, n_white = 0;
  void* render_spill = nullptr;  // per env: listed words past the LDS list (dtrender.hip)
  void* render_sched = nullptr;  // render_kernel's dispatch order state (dtrender.hip)
  uint32_t render_launches = 0;  // dt_render launches (the order's double-buffer parity)
  // the last render launch that used the dispatch-order state: its stream and
  // an event recorded after it (a render on another stream waits for it)
  hipEvent_t render_done = nullptr;
  hipStream_t render_stream = nullptr;
  bool render_pending = false;
  std::string err;
};

// Launch entry points run on the handle's GPU whatever the calling thread's
// current device is (a VecEnv on cuda:1 called from a thread whose current
// device is 0); the caller's current device is restored on return.
struct DevGuard {
  int prev = -1;
  explicit DevGuard(int device) {
    if (hipGetDevice(&prev) == hipSuccess && prev != device) {
      if (hipSetDevice(device) != hipSuccess) prev = -1;
    } else {
      prev = -1;
    }
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DevGuard(const DevGuard&) = delete;
  DevGuard& operator=(const DevGuard&) = delete;
};

// record a failed HIP call in the handle and return DT_E_HIP
#define HIP_OR_FAIL(h, expr)                                                   \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      (h)->err = std::string(#expr) + ": " + hipGetErrorString(_e);             \
      return DT_E_HIP;                                                         \
    }                                                                          \
  } while (0)

// dtrender.hip: lane-marking polylines of the map + default line params
int dt_render_init(dt_handle* h, const dt_map* map);
void dt_render_free(dt_handle* h);


