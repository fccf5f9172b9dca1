// tools/sync_wait_probe.cpp -- host wait after a C5-step launch, from C++.
//
// The host-driven protocol (the library's default, comm.h:186-206) waits
// twice per pipeline step: the transport stream's copies, then the step's
// batched reduction (hiccl_reduce_plan_sync = hipStreamSynchronize, as the
// reference's Compute<T>::wait, compute.h:107-117).  This probe times one
// C5 step's plan (four 2-input and one 4-input compute of 2^18 f32) as
// launch + wait on the host clock, 2000 steps per variant, interleaved in
// rounds, with the wait done by
//   sync        hipStreamSynchronize (what the library does),
//   event_sync  hipEventRecord after the launch + hipEventSynchronize,
//   query_spin  hipStreamQuery in a loop,
//   event_spin  hipEventRecord + hipEventQuery in a loop,
// and the kernel alone by HIP events.  argv[1] = "spin" sets
// hipDeviceScheduleSpin before the context exists (argv[1] = "yield":
// hipDeviceScheduleYield, "block": hipDeviceScheduleBlockingSync, anything
// else: the runtime's default).  One JSON line per variant.
//   build: see tools/sync_wait_probe.sh
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../include/hiccl_reduce.h"

static void ok(int e, const char *what) {
  if (e) {
    std::fprintf(stderr, "%s failed: %d %s\n", what, e, hiccl_last_error());
    std::exit(1);
  }
}

int main(int argc, char **argv) {
  const std::string sched = argc > 1 ? argv[1] : "default";
  unsigned flags = sched == "spin" ? hipDeviceScheduleSpin
                   : sched == "yield" ? hipDeviceScheduleYield
                   : sched == "block" ? hipDeviceScheduleBlockingSync
                                      : hipDeviceScheduleAuto;
  if (sched != "default") ok(hipSetDeviceFlags(flags), "hipSetDeviceFlags");
  ok(hipSetDevice(0), "hipSetDevice");
  const size_t c = 1 << 18;
  std::vector<float *> bufs(12), outs(5);
  for (auto &b : bufs) {
    ok(hipMalloc((void **)&b, c * 4), "hipMalloc");
    ok(hiccl_fill_uniform(HICCL_FLOAT32, b, c, 1234, (uint32_t)(&b - bufs.data()), 0, nullptr), "fill");
  }
  for (auto &o : outs) ok(hipMalloc((void **)&o, c * 4), "hipMalloc");
  hiccl_reduce_plan_t *plan = nullptr;
  ok(hiccl_reduce_plan_create(&plan, HICCL_FLOAT32, 0), "plan_create");
  for (int j = 0; j < 4; j++) {
    const void *in[2] = {bufs[2 * j], bufs[2 * j + 1]};
    ok(hiccl_reduce_plan_add(plan, outs[j], in, 2, c), "plan_add");
  }
  const void *in4[4] = {bufs[8], bufs[9], bufs[10], bufs[11]};
  ok(hiccl_reduce_plan_add(plan, outs[4], in4, 4, c), "plan_add");
  hipStream_t s;
  ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "stream");
  hipEvent_t ev, a, b;
  ok(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "event");
  ok(hipEventCreate(&a), "event");
  ok(hipEventCreate(&b), "event");
  for (int i = 0; i < 50; i++) {
    ok(hiccl_reduce_plan_enqueue(plan, s), "enqueue");
    ok(hipStreamSynchronize(s), "sync");
  }
  const char *names[4] = {"sync", "event_sync", "query_spin", "event_spin"};
  std::vector<std::vector<double>> res(4);
  const int steps = 2000;
  for (int round = 0; round < 5; round++) {
    for (int v = 0; v < 4; v++) {
      std::vector<double> t(steps);
      for (int i = 0; i < steps; i++) {
        const auto t0 = std::chrono::steady_clock::now();
        ok(hiccl_reduce_plan_enqueue(plan, s), "enqueue");
        if (v == 0) {
          ok(hipStreamSynchronize(s), "sync");
        } else if (v == 1) {
          ok(hipEventRecord(ev, s), "record");
          ok(hipEventSynchronize(ev), "event sync");
        } else if (v == 2) {
          hipError_t e;
          while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
          }
          ok(e, "query");
        } else {
          ok(hipEventRecord(ev, s), "record");
          hipError_t e;
          while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
          }
          ok(e, "event query");
        }
        t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      }
      std::sort(t.begin(), t.end());
      res[v].push_back(t[steps / 2]);
      res[v].push_back(t[steps / 10]);
      res[v].push_back(t[steps * 9 / 10]);
    }
  }
  // the kernel alone (events around 200 back-to-back launches)
  ok(hipEventRecord(a, s), "record");
  for (int i = 0; i < 200; i++) ok(hiccl_reduce_plan_enqueue(plan, s), "enqueue");
  ok(hipEventRecord(b, s), "record");
  ok(hipEventSynchronize(b), "sync");
  float ms = 0;
  ok(hipEventElapsedTime(&ms, a, b), "elapsed");
  for (int v = 0; v < 4; v++) {
    std::vector<double> med, p10, p90;
    for (size_t r = 0; r < res[v].size(); r += 3) {
      med.push_back(res[v][r]);
      p10.push_back(res[v][r + 1]);
      p90.push_back(res[v][r + 2]);
    }
    std::sort(med.begin(), med.end());
    std::sort(p10.begin(), p10.end());
    std::sort(p90.begin(), p90.end());
    std::printf("{\"probe\": \"host_wait_cpp\", \"schedule\": \"%s\", \"wait\": \"%s\", \"median_us\": %.3f, "
                "\"p10_us\": %.3f, \"p90_us\": %.3f, \"kernel_queued_us\": %.3f, \"store_policy\": %d}\n",
                sched.c_str(), names[v], med[med.size() / 2], p10[p10.size() / 2], p90[p90.size() / 2],
                ms * 1e3 / 200, hiccl_reduce_plan_store_policy(plan));
  }
  hiccl_reduce_plan_destroy(plan);
  return 0;
}
