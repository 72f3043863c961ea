// launch_fan.h — host-side fan-out of one logical launch over several HIP streams.
//
// The band and NMPC kernels are issued as several class launches (QP size x LDS occupancy), each
// spanning the whole batch.  Issued back to back on one stream they serialise, and a class whose
// workgroups need 80-160 KB of LDS then holds one wave per CU while three SIMDs idle.  The fan
// forks the class launches over the caller's stream plus up to kFanAux auxiliary streams
// (event-joined back into the caller's stream, so the caller still synchronises on its own
// stream only) and lets the dispatcher co-schedule light classes beside heavy ones.
#pragma once
#include <hip/hip_runtime.h>

namespace mpct {

constexpr int kFanAux = 3;  // + the caller's stream = 4 (GPU_MAX_HW_QUEUES on the pool is 4)

struct LaunchFan {
  int dev = -1;
  hipStream_t aux[kFanAux] = {};
  hipEvent_t fork = nullptr;
  hipEvent_t join[kFanAux] = {};
  bool ready = false;

  // create the streams / events on the current device (idempotent); false on failure
  bool init(int device) {
    if (ready && dev == device) return true;
    release();
    for (int k = 0; k < kFanAux; ++k)
      if (hipStreamCreateWithFlags(&aux[k], hipStreamNonBlocking) != hipSuccess) return false;
    if (hipEventCreateWithFlags(&fork, hipEventDisableTiming) != hipSuccess) return false;
    for (int k = 0; k < kFanAux; ++k)
      if (hipEventCreateWithFlags(&join[k], hipEventDisableTiming) != hipSuccess) return false;
    dev = device;
    ready = true;
    return true;
  }
  void release() {
    for (int k = 0; k < kFanAux; ++k) {
      if (aux[k]) (void)hipStreamDestroy(aux[k]);
      if (join[k]) (void)hipEventDestroy(join[k]);
      aux[k] = nullptr;
      join[k] = nullptr;
    }
    if (fork) (void)hipEventDestroy(fork);
    fork = nullptr;
    ready = false;
  }
};

// One fan-out: stream(k) for the k-th class launch (k = 0 on the caller's stream), join() at the end.
struct FanScope {
  LaunchFan* fan;
  hipStream_t main;
  bool used[kFanAux] = {};
  bool forked = false;
  // the fork point is recorded before any class launch: an auxiliary stream must not wait for a
  // class launch already queued on the caller's stream
  FanScope(LaunchFan* f, hipStream_t s) : fan(f && f->ready ? f : nullptr), main(s) {
    if (fan) forked = hipEventRecord(fan->fork, main) == hipSuccess;
    if (!forked) fan = nullptr;
  }
  hipStream_t stream(int k) {
    if (!fan || k % (kFanAux + 1) == 0) return main;
    const int a = k % (kFanAux + 1) - 1;
    if (!used[a]) {
      (void)hipStreamWaitEvent(fan->aux[a], fan->fork, 0);
      used[a] = true;
    }
    return fan->aux[a];
  }
  void join() {
    if (!fan) return;
    for (int a = 0; a < kFanAux; ++a)
      if (used[a]) {
        (void)hipEventRecord(fan->join[a], fan->aux[a]);
        (void)hipStreamWaitEvent(main, fan->join[a], 0);
      }
  }
};

}  // namespace mpct
