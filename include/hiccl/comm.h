// include/hiccl/comm.h -- HiCCL::Comm<T>, the persistent communicator
// (reference: source/comm.h, source/init.h).
//
// Epochs of REDUCE/BROADCAST primitives separated by fences; init() turns
// them into a pipeline of steps (init.h:2-76 + command.h implement);
// run() executes it (comm.h:181-206): every library's transport starts, then
// in reverse library order each transport completes and that library's
// compute is launched, then every compute completes.
//
// Schedule<T> is the pure part (primitives + parameters -> merged steps for
// one rank), so the factorization can be produced for any rank of any
// machine size without MPI (tests/cpp/plan_dump.cpp).
#ifndef HICCL_COMM_H
#define HICCL_COMM_H

#include <pthread.h>

#include <algorithm>

#include <cstdio>
#include <cstdlib>
#include <list>
#include <string>
#include <vector>

#include "command.h"
#include "compute.h"
#include "plan.h"

namespace HiCCL {

enum pattern { all, others };

template <typename T>
struct Schedule {
  std::vector<std::vector<BROADCAST<T>>> bcast_epoch;
  std::vector<std::vector<REDUCE<T>>> reduce_epoch;
  std::vector<int> hierarchy;
  std::vector<CommBench::library> library;
  int numstripe = 1, ringnodes = 1, pipedepth = 1;

  void fence() {
    bcast_epoch.emplace_back();
    reduce_epoch.emplace_back();
  }
  void reduce(T *sb, size_t so, T *rb, size_t ro, size_t count, std::vector<int> ids, int recvid) {
    reduce_epoch.back().emplace_back(sb, so, rb, ro, count, std::move(ids), recvid);
  }
  void bcast(T *sb, size_t so, T *rb, size_t ro, size_t count, int sendid, std::vector<int> ids) {
    bcast_epoch.back().emplace_back(sb, so, rb, ro, count, sendid, std::move(ids));
  }

  // comm.h:160-179: groupsize[L-1] = h[L-1], groupsize[i] = groupsize[i+1]*h[i],
  // then groupsize[0] = numproc / ringnodes.
  std::vector<int> groupsizes(int np) const {
    const int L = (int)hierarchy.size();
    std::vector<int> g(L);
    g[L - 1] = hierarchy[L - 1];
    for (int i = L - 2; i >= 0; i--) g[i] = g[i + 1] * hierarchy[i];
    g[0] = np / ringnodes;
    return g;
  }

  // init.h:2-76 for rank `me` of `np`: per epoch, multicasts then
  // reductions, each split into pipedepth batches; returns the per-batch
  // level lists (coll_batch) and the planner's memory counters.
  std::vector<CollList<T>> factorize(Planner<T> &P) const {
    const int np = P.np, L = (int)hierarchy.size();
    std::vector<int> gs = groupsizes(np), gt = gs;
    gt[0] = np;
    std::vector<CollList<T>> batches(pipedepth);
    for (size_t e = 0; e < reduce_epoch.size(); e++) {
      if (!bcast_epoch[e].empty()) {
        auto parts = partition(bcast_epoch[e], pipedepth);
        for (int b = 0; b < pipedepth; b++) {
          auto split = P.stripe(numstripe, parts[b]);
          typename Planner<T>::Pool pool;
          P.reduce_tree(1, gt.data(), &library[L - 1], split, 0, batches[b], pool);
          std::vector<BROADCAST<T>> intra;
          P.bcast_ring(gs[0], library[0], parts[b], intra, batches[b]);
          P.bcast_tree(L, gt.data(), library.data(), intra, 1, batches[b]);
        }
      }
      if (!reduce_epoch[e].empty()) {
        auto parts = partition(reduce_epoch[e], pipedepth);
        for (int b = 0; b < pipedepth; b++) {
          auto merge = P.stripe(numstripe, parts[b]);
          std::vector<REDUCE<T>> intra;
          P.reduce_ring(L, gs.data(), library.data(), parts[b], intra, batches[b]);
          P.bcast_tree(L, gt.data(), library.data(), merge, 1, batches[b]);
        }
      }
    }
    return batches;
  }
};

template <typename T>
class Comm {
 public:
  // PIPELINE (comm.h:154-156): one list of commands per library
  std::vector<std::list<Command<T>>> command_batch;
  std::vector<CollList<T>> coll_batch;
  std::vector<CommBench::library> libs;

  Comm() {
    sch.hierarchy = {CommBench::numproc};
    sch.library = {CommBench::MPI};
    add_fence();  // epoch 0 (comm.h:120-128)
  }
  Comm(const Comm &) = delete;  // owns its schedule buffers, plans and streams
  Comm &operator=(const Comm &) = delete;

  // ------------------------------------------------------------ setters --
  void set_hierarchy(std::vector<int> hierarchy, std::vector<CommBench::library> library) {
    if (hierarchy.size() != library.size() || hierarchy.empty()) {
      if (CommBench::myid == CommBench::printid) std::printf("hierarchy and library must have the same size!\n");
      return;
    }
    sch.hierarchy = hierarchy;
    sch.library = library;
  }
  void set_pipedepth(int d) { sch.pipedepth = d < 1 ? 1 : d; }
  void set_numstripe(int s) { sch.numstripe = s < 1 ? 1 : s; }
  void set_ringnodes(int r) { sch.ringnodes = r < 1 ? 1 : r; }
  // Stream-ordered execution (HIP port, all ranks on one node, one GPU per
  // rank): every step's transfers, their ready/done signalling and its
  // compute are enqueued on the rank's stream and run() synchronises once at
  // the end.  Opt-in (HICCL_STREAM_ORDERED=1 or this setter).  When ranks
  // share a device, init() falls back to host-driven mode and says so: the
  // spinning waits of co-resident ranks can hold the device's hardware
  // queues while a peer's queue is not mapped.
  // `force` (HICCL_STREAM_ORDERED=force) keeps the mode anyway -- for
  // single-GPU rehearsals with few hardware queues per process
  // (GPU_MAX_HW_QUEUES), not for production.
  void set_stream_ordered(bool on, bool force = false) { stream_req = on ? (force ? 2 : 1) : 0; }
  // Fused gather + reduce (HIP port, IPC / IPC_get levels): a transfer whose
  // receive buffer only feeds a reduction of the same step is not copied;
  // the reduction kernel reads the sender's buffer over xGMI in place.
  // Opt-in (HICCL_FUSED_GATHER=1 or this setter); results are identical.
  void set_fused_gather(bool on) { fuse_req = on ? 1 : 0; }
  // hipGraph replay of stream-ordered runs (HIP port; needs stream-ordered
  // mode): the first run() executes eagerly (uploads every plan), the second
  // captures the whole enqueued pipeline into a graph, and every run()
  // replays it -- one hipGraphLaunch instead of a few launches per step.
  // The signal epochs come from a device counter the graph bumps first
  // (hiccl_signal_wait_dev).  Opt-in (HICCL_GRAPH=1 or this setter); every
  // rank must agree (init reduces the choice).
  void set_graph(bool on) { graph_req = on ? 1 : 0; }
  bool graph_mode() const { return graphed; }
  void set_endpoints(T *sb, size_t sc, T *rb, size_t rc) {
    sendbuf = sb;
    sendcount = sc;
    recvbuf = rb;
    recvcount = rc;
  }

  void print_parameters() const {
    if (CommBench::myid != CommBench::printid) return;
    std::printf("**************** HiCCL PARAMETERS\n%zu-level hierarchy:\n", sch.hierarchy.size());
    for (size_t i = 0; i < sch.hierarchy.size(); i++)
      std::printf("  level %zu factor: %d library: %s\n", i, sch.hierarchy[i], CommBench::lib_name(sch.library[i]));
    std::printf("numstripe: %d\nringnodes: %d\npipedepth: %d\n", sch.numstripe, sch.ringnodes, sch.pipedepth);
    std::printf("sendbuf: %p, sendcount %zu\nrecvbuf: %p, recvcount %zu\n", (void *)sendbuf, sendcount,
                (void *)recvbuf, recvcount);
    std::printf("*********************************\n");
  }

  // ------------------------------------------------------- primitives ----
  void add_fence() {
    sch.fence();
    numepoch++;
  }

  // comm.h:131-143 (add_bcast) -- recvids as a list, a rank, or a pattern
  void add_bcast(T *sb, size_t so, T *rb, size_t ro, size_t count, int sendid, std::vector<int> &recvids) {
    sch.bcast(sb, so, rb, ro, count, sendid, recvids);
  }
  void add_bcast(T *sb, size_t so, T *rb, size_t ro, size_t count, int sendid, int recvid) {
    sch.bcast(sb, so, rb, ro, count, sendid, expand_ids(recvid, CommBench::numproc, sendid));
  }
  void add_bcast(T *sb, size_t so, T *rb, size_t ro, size_t count, int sendid, pattern p) {
    add_bcast(sb, so, rb, ro, count, sendid, p == others ? -1 : CommBench::numproc);
  }

  // comm.h:144-156 (add_reduce) -- sendids as a list, a rank, or a pattern
  void add_reduce(T *sb, size_t so, T *rb, size_t ro, size_t count, std::vector<int> &sendids, int recvid) {
    sch.reduce(sb, so, rb, ro, count, sendids, recvid);
  }
  void add_reduce(T *sb, size_t so, T *rb, size_t ro, size_t count, int sendid, int recvid) {
    sch.reduce(sb, so, rb, ro, count, expand_ids(sendid, CommBench::numproc, recvid), recvid);
  }
  void add_reduce(T *sb, size_t so, T *rb, size_t ro, size_t count, pattern p, int recvid) {
    add_reduce(sb, so, rb, ro, count, p == others ? -1 : CommBench::numproc, recvid);
  }

  // README.md:33,38 spellings (offset 0).
  void add_reduction(T *sb, T *rb, size_t count, pattern p, int recvid) { add_reduce(sb, 0, rb, 0, count, p, recvid); }
  void add_reduction(T *sb, T *rb, size_t count, int sendid, int recvid) { add_reduce(sb, 0, rb, 0, count, sendid, recvid); }
  void add_reduction(T *sb, T *rb, size_t count, std::vector<int> &sendids, int recvid) {
    add_reduce(sb, 0, rb, 0, count, sendids, recvid);
  }
  void add_multicast(T *sb, T *rb, size_t count, int sendid, pattern p) { add_bcast(sb, 0, rb, 0, count, sendid, p); }
  void add_multicast(T *sb, T *rb, size_t count, int sendid, int recvid) { add_bcast(sb, 0, rb, 0, count, sendid, recvid); }
  void add_multicast(T *sb, T *rb, size_t count, int sendid, std::vector<int> &recvids) {
    add_bcast(sb, 0, rb, 0, count, sendid, recvids);
  }

  // ---------------------------------------------------------------- init --
  // README.md:48 spelling: init(hierarchy, lib, numstripe, ring, pipeline)
  void init(std::vector<int> hierarchy, std::vector<CommBench::library> lib, int numstripe, int ring, int pipeline) {
    set_hierarchy(hierarchy, lib);
    set_numstripe(numstripe);
    set_ringnodes(ring);
    set_pipedepth(pipeline);
    init();
  }

  void init() {
    if (CommBench::myid == CommBench::printid) print_parameters();
    MPI_Barrier(CommBench::comm_mpi);
    const double t0 = MPI_Wtime();
    Planner<T> P(CommBench::myid, CommBench::numproc, [this](size_t n) {
      T *p = nullptr;
      CommBench::allocate(p, n);
      owned.push_back(p);
      return p;
    });
    coll_batch = sch.factorize(P);
    libs = libraries_used(coll_batch);
    steps = merge_steps(coll_batch, libs, 1);
#ifndef HICCL_PORT_HOST
    device_ranks = CommBench::ranks_on_my_device();
    shared_device = CommBench::ranks_share_device();
    if (std::find(libs.begin(), libs.end(), CommBench::XCCL) != libs.end()) {
      xccl = CommBench::xccl_setup(shared_device);
      if (!xccl && CommBench::myid == CommBench::printid)
        std::printf("HiCCL: XCCL levels run on the IPC path (%s)\n",
#ifdef HICCL_WITH_RCCL
                    !CommBench::xccl_rccl_requested() ? "RCCL is opt-in: HICCL_XCCL=rccl"
                                                      : "ranks share a GPU: RCCL needs one GPU per rank"
#else
                    "built without HICCL_WITH_RCCL"
#endif
        );
    }
#endif
    streamed = want_stream_mode();
    fused = want_fused();
    graphed = streamed && want_graph();
    if (graphed && xccl) {  // RCCL groups are not recorded into the replay graph
      graphed = false;
      if (CommBench::myid == CommBench::printid) std::printf("HiCCL: graph replay off (XCCL level on RCCL)\n");
    }
    CommBench::stream_ordered = streamed;
    command_batch = instantiate(steps, libs, fused);
    CommBench::stream_ordered = false;
#ifndef HICCL_PORT_HOST
    programs = streamed && want_programs();
    if (streamed) {  // one flag pair per registered transfer, every rank the same layout
      size_t total = 0;
      for (auto &lst : command_batch)
        for (auto &c : lst) total += c.comm->size();
      flags.create(2 * total);
      size_t base = 0;
      for (auto &lst : command_batch)
        for (auto &c : lst) {
          c.comm->bind(&flags, base);
          base += c.comm->size();
        }
    }
#endif
    buffsize = P.buffsize;
    recycle = P.recycle;
    reuse = P.reuse;
    MPI_Barrier(CommBench::comm_mpi);  // nobody runs before every rank's handles are exchanged
    report_memory();
    if (CommBench::myid == CommBench::printid)
      std::printf("initialization time: %e seconds (%zu steps, %zu libraries, %s%s%s%s)\n", MPI_Wtime() - t0,
                  steps.size(), libs.size(), streamed ? "stream-ordered" : "host-driven", graphed ? ", graph replay" : "",
                  fused ? ", fused gather" : "", xccl ? ", XCCL on RCCL" : "");
#ifndef HICCL_PORT_HOST
    if (streamed && CommBench::myid == CommBench::printid)
      std::printf("stream-ordered protocol: %s tokens, %s\n",
                  hiccl_token_mode() == HICCL_TOKENS_LIGHT ? "light (relaxed, HICCL_PROG_FENCES=light)"
                                                           : "fenced (release / acquire)",
                  programs ? "step programs (HICCL_STEP_PROGRAM=1)" : "one launch per element");
    if (programs && CommBench::myid == CommBench::printid) std::printf("step programs: token phases folded into the step's launches\n");
#endif
  }

  bool xccl_on_rccl() const { return xccl; }
  bool shares_device() const { return shared_device; }  // two or more ranks drive one GPU (init)

  bool stream_ordered() const { return streamed; }
  bool fused_gather() const { return fused; }
#ifndef HICCL_PORT_HOST
  bool step_program_mode() const { return programs; }
#endif

  // ----------------------------------------------------------------- run --
  // comm.h:181-206
  void run() {
#ifndef HICCL_PORT_HOST
    if (streamed) return run_streamed();
#endif
    const size_t nl = command_batch.size();
    std::vector<typename std::list<Command<T>>::iterator> it(nl);
    for (size_t i = 0; i < nl; i++) it[i] = command_batch[i].begin();
    if (nl == 0) return;
    if (timing) return run_timed(it);
    while (it[0] != command_batch[0].end()) {  // every library has one command per step
      for (size_t i = 0; i < nl; i++) it[i]->comm->start();
      for (size_t i = nl; i-- > 0;) {
        it[i]->comm->wait();
        it[i]->compute->start();
      }
      for (size_t i = 0; i < nl; i++) it[i]->compute->wait();
      for (size_t i = 0; i < nl; i++) {
        it[i]->comm->finish();  // fused transfers: release the senders' buffers
        ++it[i];
      }
    }
  }

  // Host wall time of run() split by what the host waits on, per step, in
  // comm.h:186-206's order: host-driven -- transport start, transport wait,
  // compute launch, compute wait (comm.h:195-204), and the fused transfers'
  // release; stream-ordered -- enqueueing the pipeline (or launching its
  // graph) and the one synchronisation at the end.  Seconds, summed over the
  // runs since set_step_timing(true); `steps` = pipeline steps per run.
  struct StepSplit {
    double transport_start = 0, transport_wait = 0, compute_launch = 0, compute_wait = 0, finish = 0;
    double enqueue = 0, sync = 0;
    size_t runs = 0, steps = 0;
  };
  void set_step_timing(bool on) {
    timing = on;
    split = StepSplit{};
    split.steps = steps.size();
  }
  const StepSplit &step_split() const { return split; }

  // comm.h:208-212
  void run(T *sb, T *rb) {
    CommBench::memcpyD2D(sendbuf, sb, sendcount);
    run();
    CommBench::memcpyD2D(rb, recvbuf, recvcount);
  }

  // comm.h:214-227: nonblocking run on a pthread bound to the rank's device.
  void start() {
    if (pthread_create(&thread, nullptr, &Comm<T>::run_async, this) != 0)
      CommBench::die("Comm::start", "pthread_create failed");
    running = true;
  }
  void wait() {
    if (running) pthread_join(thread, nullptr);
    running = false;
  }

  // comm.h:229-271: measure every command of the pipeline in step order.
  void measure(int warmup, int numiter, size_t count) {
    if (CommBench::myid == CommBench::printid)
      std::printf("command_batch size %zu\ncommandlist size %zu\n", command_batch.size(),
                  command_batch.empty() ? (size_t)0 : command_batch[0].size());
    MPI_Barrier(CommBench::comm_mpi);
    const size_t nl = command_batch.size();
    if (!nl) return;
    std::vector<typename std::list<Command<T>>::iterator> it(nl);
    for (size_t i = 0; i < nl; i++) it[i] = command_batch[i].begin();
    while (it[0] != command_batch[0].end()) {
      if (CommBench::myid == CommBench::printid) std::printf("******************** MEASURE COMMANDS ********************\n");
      for (size_t i = 0; i < nl; i++) {
        it[i]->measure(warmup, numiter, count);
        ++it[i];
      }
    }
  }

  // Per-step structure (the reference's report_pipeline, coll.h:97-152).
  void report() const {
    if (CommBench::myid != CommBench::printid) return;
    std::printf("pipeline: %zu steps x %zu libraries\n", steps.size(), libs.size());
    for (size_t s = 0; s < steps.size(); s++) {
      std::printf("step %zu:\n", s);
      for (auto &c : steps[s])
        if (!c.empty()) {
          std::printf("  ");
          c.report(CommBench::numproc);
        }
    }
  }

#ifndef HICCL_PORT_HOST
  // Kernel time of this rank's batched compute per step: HIP events around
  // the step's plan launch alone on the compute stream, median of `reps`
  // (after one warm launch), for every step in which this rank computes.
  // Measurement only -- it overwrites the steps' outputs, so run it before
  // (not between) the runs whose results are checked.  Returns
  // {milliseconds, algorithmic bytes} per step.
  std::vector<std::pair<double, size_t>> compute_kernel_times(int reps) {
    std::vector<std::pair<double, size_t>> out;
    CommBench::setup_gpu();
    hipStream_t s = compute_stream();
    hipEvent_t a, b;
    CommBench::hip_check(hipEventCreate(&a), "hipEventCreate");
    CommBench::hip_check(hipEventCreate(&b), "hipEventCreate");
    for (auto &lst : command_batch)
      for (auto &c : lst) {
        if (!c.compute->numcomp) continue;
        c.compute->launch(s);  // warm (and the plan's one-time upload)
        std::vector<float> t;
        for (int r = 0; r < std::max(reps, 1); r++) {
          CommBench::hip_check(hipEventRecord(a, s), "hipEventRecord");
          c.compute->launch(s);
          CommBench::hip_check(hipEventRecord(b, s), "hipEventRecord");
          CommBench::hip_check(hipEventSynchronize(b), "hipEventSynchronize");
          float ms = 0;
          CommBench::hip_check(hipEventElapsedTime(&ms, a, b), "hipEventElapsedTime");
          t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        out.emplace_back((double)t[t.size() / 2], c.compute->bytes());
      }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return out;
  }
#endif

  size_t numsteps() const { return steps.size(); }
  const std::vector<std::vector<Coll<T>>> &plan() const { return steps; }
  const Schedule<T> &schedule() const { return sch; }

  size_t buffsize = 0, recycle = 0, reuse = 0;

 private:
  Schedule<T> sch;
  int numepoch = 0;
  T *sendbuf = nullptr, *recvbuf = nullptr;
  size_t sendcount = 0, recvcount = 0;
  std::vector<std::vector<Coll<T>>> steps;
  pthread_t thread{};
  bool running = false;

  bool timing = false;
  StepSplit split;

  // run() with the host wall split recorded (set_step_timing): the same calls
  // in the same order, a clock read between them.
  template <class It>
  void run_timed(std::vector<It> &it) {
    const size_t nl = it.size();
    double t = MPI_Wtime();
    auto lap = [&t](double &acc) {
      const double u = MPI_Wtime();
      acc += u - t;
      t = u;
    };
    while (it[0] != command_batch[0].end()) {
      for (size_t i = 0; i < nl; i++) it[i]->comm->start();
      lap(split.transport_start);
      for (size_t i = nl; i-- > 0;) {
        it[i]->comm->wait();
        lap(split.transport_wait);
        it[i]->compute->start();
        lap(split.compute_launch);
      }
      for (size_t i = 0; i < nl; i++) it[i]->compute->wait();
      lap(split.compute_wait);
      for (size_t i = 0; i < nl; i++) {
        it[i]->comm->finish();
        ++it[i];
      }
      lap(split.finish);
    }
    split.runs++;
  }

  int stream_req = -1;  // -1: decide from the environment and the node layout; 2: forced
  bool streamed = false;
  bool shared_device = false;  // two or more ranks drive one GPU
  int device_ranks = 1;        // ranks driving this rank's GPU (this one included)
  bool xccl = false;           // XCCL levels run on RCCL
  int fuse_req = -1;  // -1: HICCL_FUSED_GATHER
  bool fused = false;
  int graph_req = -1;  // -1: HICCL_GRAPH
  bool graphed = false;
#ifndef HICCL_PORT_HOST
  CommBench::FlagSpace flags;

  // Same order as run(), all of it enqueued on one stream: per step, every
  // library's transport (ready signal, wait, copies, done signal, wait),
  // then the computes in reverse library order; one synchronisation.
  void run_streamed() {
    CommBench::setup_gpu();
    hipStream_t s = CommBench::transport_stream();
    if (command_batch.empty()) return;
    const double t0 = timing ? MPI_Wtime() : 0.0;
    if (graphed && ran_eager) {
      if (gexec && !epochs_match()) drop_graph();  // eager executions since (measure): re-record
      if (!gexec) capture(s);
      CommBench::hip_check(hipGraphLaunch(gexec, s), "run: hipGraphLaunch");
      for_each_comm([](CommBench::Comm<T> &c) { c.replayed(); });
      replays++;
    } else {
      enqueue_pipeline(s);
      ran_eager = true;
    }
    CommBench::flush_signals();
    const double t1 = timing ? MPI_Wtime() : 0.0;
    CommBench::hip_check(hipStreamSynchronize(s), "run: stream sync");
    if (timing) {
      split.enqueue += t1 - t0;
      split.sync += MPI_Wtime() - t1;
      split.runs++;
    }
    if (*flags.err) CommBench::die("run", "stream-ordered signal timed out (a peer never signalled)");
  }

  void enqueue_pipeline(hipStream_t s) {
    if (programs) return enqueue_programs(s);
    const size_t nl = command_batch.size();
    std::vector<typename std::list<Command<T>>::iterator> it(nl);
    for (size_t i = 0; i < nl; i++) it[i] = command_batch[i].begin();
    while (it[0] != command_batch[0].end()) {
      for (size_t i = 0; i < nl; i++) it[i]->comm->enqueue(s);
      for (size_t i = nl; i-- > 0;) it[i]->compute->launch(s);
      for (size_t i = 0; i < nl; i++) {
        it[i]->comm->enqueue_tail(s);
        ++it[i];
      }
    }
    CommBench::flush_signals();  // (the last step's done tokens)
  }

  // Programs (HICCL_STEP_PROGRAM=1; stream-ordered mode, opt-in,
  // want_programs()): the
  // first stream-ordered run() records the enqueue sequence above -- per
  // step every library's ready tokens, copies and done tokens, the computes
  // in reverse library order, the fused transfers' done tokens -- as a list
  // of hiccl_programs, each a group of token phases folded into the launch
  // of the copy or compute batch that follows it (include/hiccl_reduce.h);
  // later runs launch the list: no separate signal/wait kernels (reference
  // order: comm.h:195-204's transport wait -> compute start -> compute
  // wait).  Every transport still counts the run (advance()), and each
  // phase's epoch is read from its transport at launch.
  std::vector<CommBench::StepRecorder::Launch> prog_launches;
  bool prog_recorded = false;
  bool programs = false;
  bool in_capture = false;

  void enqueue_programs(hipStream_t s) {
    if (!prog_recorded) {  // never inside a capture: the first run is eager
      if (in_capture) CommBench::die("program", "the pipeline was first met inside a graph capture");
      CommBench::flush_signals();
      CommBench::StepRecorder rec;
      rec.dtype = dtype_of<T>();
      rec.device = CommBench::mydevice;
      // a program's workgroups wait on the GPU for its phases; ranks sharing
      // the GPU (single-GPU rehearsals only) split its workgroup slots so
      // every rank's kernels stay resident while the others wait for them
      rec.max_wg = device_ranks > 1 ? program_grid_share() : 0;
      // A step's transports in the reference's order (comm.h:188-204: every
      // transport starts, then each is waited for): all ready phases, all
      // copies as ONE batch, all done phases, then the computes as one batch
      // -- two launches per step (the fused transfers' tail phases ride in
      // the next step's first program).
      rec.join_all_copies = true;
      CommBench::step_recorder() = &rec;
      const size_t nl = command_batch.size();
      std::vector<typename std::list<Command<T>>::iterator> it(nl);
      for (size_t i = 0; i < nl; i++) it[i] = command_batch[i].begin();
      while (it[0] != command_batch[0].end()) {
        for (size_t i = 0; i < nl; i++) it[i]->comm->enqueue_pre(s);
        for (size_t i = 0; i < nl; i++) it[i]->comm->enqueue_copies(s);
        for (size_t i = 0; i < nl; i++) it[i]->comm->enqueue_post(s);
        for (size_t i = nl; i-- > 0;) it[i]->compute->launch(s);
        rec.end_step();
        for (size_t i = 0; i < nl; i++) {
          it[i]->comm->enqueue_tail(s);
          ++it[i];
        }
      }
      CommBench::flush_signals();
      rec.close();
      CommBench::step_recorder() = nullptr;
      prog_launches = std::move(rec.launches);
      prog_recorded = true;
    } else {
      for_each_comm([](CommBench::Comm<T> &c) { c.advance(); });  // the run counts, as enqueue() would
    }
    std::vector<uint32_t> epochs;
    for (auto &L : prog_launches) {
      epochs.resize(L.epoch_of.size());
      for (size_t i = 0; i < epochs.size(); i++) epochs[i] = L.epoch_of[i]();
      if (hiccl_program_launch(L.prog, epochs.data(), in_capture ? graph_ctr : nullptr, flags.err,
                               CommBench::signal_timeout(), s))
        CommBench::die("program", hiccl_last_error());
    }
  }

  int program_grid_share() const {
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, CommBench::mydevice) != hipSuccess) {
      (void)hipGetLastError();
      cus = 256;
    }
    return std::max(8, cus / device_ranks);
  }

  // Default: OFF (hiccl_step_program_default(); HICCL_STEP_PROGRAM=1, yes,
  // on or true opts in, any other value stays off and is named on stderr),
  // whatever the device layout.  Programs were measured only with ranks
  // sharing one GPU, where they lose (a program's workgroups wait on the
  // device for the peer's token while the peer's kernels need that device to
  // produce it: 2 ranks, pipedepth 128, 64 MiB/rank, graph + fused 2.67-2.93
  // ms with programs vs 1.57-1.58 without, profiles/r03i_c5_prog_ab.jsonl),
  // and in a one-process enqueue probe, where they win (15.2 vs 22.1 us per
  // step, profiles/r03g_progstep.jsonl).  With one GPU per rank a program's
  // gate-waiting grid also occupies every CU while ranks are out of step, so
  // the per-element launches the GPU suite verifies stay the default until an
  // 8-GPU run (bench.py's config-5 leg carries the A/B) decides.
  bool want_programs() {
    int on = hiccl_step_program_default();
    for (auto &lst : command_batch)
      for (auto &c : lst) on = on && c.comm->recordable();
    MPI_Allreduce(MPI_IN_PLACE, &on, 1, MPI_INT, MPI_LAND, CommBench::comm_mpi);
    return on != 0;
  }

  template <class F>
  void for_each_comm(F f) {
    for (auto &lst : command_batch)
      for (auto &c : lst) f(*c.comm);
  }

  // Record the pipeline once: replay counter bump, then the same enqueue
  // sequence with every wait reading its epoch through the counter.  The
  // plans were uploaded by the eager run; their launches take the static
  // unit schedule while the stream captures (no shared ticket counter in a
  // replayable graph).
  void capture(hipStream_t s) {
    CommBench::hip_check(hipMalloc((void **)&graph_ctr, sizeof(uint32_t)), "graph: hipMalloc counter");
    CommBench::hip_check(hipMemset(graph_ctr, 0, sizeof(uint32_t)), "graph: hipMemset counter");
    CommBench::hip_check(hipDeviceSynchronize(), "graph: sync");
    CommBench::hip_check(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal), "graph: begin capture");
    if (hiccl_counter_add(graph_ctr, 1, s)) CommBench::die("graph: counter", hiccl_last_error());
    for_each_comm([this](CommBench::Comm<T> &c) { c.begin_capture(graph_ctr); });
    in_capture = true;
    enqueue_pipeline(s);
    in_capture = false;
    for_each_comm([](CommBench::Comm<T> &c) { c.end_capture(); });
    graph_base.clear();
    for_each_comm([this](CommBench::Comm<T> &c) { graph_base.push_back(c.epoch_now()); });
    replays = 0;
    hipGraph_t g = nullptr;
    CommBench::hip_check(hipStreamEndCapture(s, &g), "graph: end capture");
    CommBench::hip_check(hipGraphInstantiate(&gexec, g, nullptr, nullptr, 0), "graph: instantiate");
    CommBench::hip_check(hipGraphDestroy(g), "graph: destroy");
  }

  // The graph's waits use (epoch at capture) + replay number: valid while no
  // eager execution (Comm::measure) advanced a transport's epoch since.
  bool epochs_match() {
    size_t i = 0;
    bool ok = true;
    for_each_comm([&](CommBench::Comm<T> &c) { ok = ok && c.epoch_now() == graph_base[i++] + replays; });
    return ok;
  }
  void drop_graph() {
    CommBench::hip_check(hipGraphExecDestroy(gexec), "graph: destroy exec");
    CommBench::hip_check(hipFree(graph_ctr), "graph: free counter");
    gexec = nullptr;
    graph_ctr = nullptr;
  }

  bool ran_eager = false;
  uint32_t *graph_ctr = nullptr;
  hipGraphExec_t gexec = nullptr;
  std::vector<uint32_t> graph_base;
  uint32_t replays = 0;

#endif

 public:
  // The schedule's receive / partial buffers are freed with the communicator
  // (the reference leaks them).  Collective: every rank first releases its
  // IPC mappings of its peers' buffers (deleting the transports; the
  // mappings are retired, see CommBench::IpcMapping), then a barrier, then
  // the buffers are freed.  Destroy the communicator before freeing the
  // buffers it was built on.
  ~Comm() {
    if (running) pthread_join(thread, nullptr);  // a start() without wait(): finish it first
#ifndef HICCL_PORT_HOST
    if (gexec) (void)hipGraphExecDestroy(gexec);
    if (graph_ctr) (void)hipFree(graph_ctr);
    if (!owned.empty() || !command_batch.empty()) (void)hipDeviceSynchronize();
    for (auto &L : prog_launches) hiccl_program_destroy(L.prog);
    prog_launches.clear();
#endif
    // the steps' transports (releasing their IPC mappings) and computes (the
    // reference never deletes them)
    for (auto &lst : command_batch)
      for (auto &c : lst) {
        delete c.comm;
        delete c.compute;
      }
    command_batch.clear();
#ifndef HICCL_PORT_HOST
    flags.close();  // peers' flag arrays
    int fin = 0;
    MPI_Finalized(&fin);
    if (!fin) MPI_Barrier(CommBench::comm_mpi);  // every peer has released its mappings of this rank's buffers
#endif
    for (T *p : owned) CommBench::free(p);
#ifndef HICCL_PORT_HOST
    if (xccl) CommBench::xccl_release();  // the last RCCL user destroys the communicator
#endif
  }

 private:
  std::vector<T *> owned;  // allocated by init() for the schedule

  bool want_graph() {
#ifdef HICCL_PORT_HOST
    return false;
#else
    int on = graph_req;
    if (on < 0) {
      const char *env = std::getenv("HICCL_GRAPH");
      on = (env && std::string(env) == "1") ? 1 : 0;
    }
    MPI_Allreduce(MPI_IN_PLACE, &on, 1, MPI_INT, MPI_LAND, CommBench::comm_mpi);
    return on != 0;
#endif
  }

  bool want_stream_mode() {
#ifdef HICCL_PORT_HOST
    return false;
#else
    int on = stream_req;
    if (on < 0) {
      const char *env = std::getenv("HICCL_STREAM_ORDERED");
      const std::string v = env ? env : "";
      on = v == "force" ? 2 : v == "1" ? 1 : 0;
    }
    MPI_Comm local;
    MPI_Comm_split_type(CommBench::comm_mpi, MPI_COMM_TYPE_SHARED, CommBench::myid, MPI_INFO_NULL, &local);
    int lsize = 0;
    MPI_Comm_size(local, &lsize);
    MPI_Comm_free(&local);
    int ok = on && lsize == CommBench::numproc && (!shared_device || on == 2);
    MPI_Allreduce(MPI_IN_PLACE, &ok, 1, MPI_INT, MPI_LAND, CommBench::comm_mpi);
    if (on && !ok && shared_device && CommBench::myid == CommBench::printid)
      std::printf("HiCCL: ranks share a GPU -- stream-ordered mode needs one GPU per rank; running host-driven "
                  "(HICCL_STREAM_ORDERED=force overrides)\n");
    return ok != 0;
#endif
  }

  bool want_fused() {
#ifdef HICCL_PORT_HOST
    return false;
#else
    int on = fuse_req;
    if (on < 0) {
      const char *env = std::getenv("HICCL_FUSED_GATHER");
      on = (env && std::string(env) == "1") ? 1 : 0;
    }
    MPI_Allreduce(MPI_IN_PLACE, &on, 1, MPI_INT, MPI_LAND, CommBench::comm_mpi);
    return on != 0;
#endif
  }

  static void *run_async(void *arg) {
    CommBench::setup_gpu();
    static_cast<Comm<T> *>(arg)->run();
    return nullptr;
  }

  // command.h:46-78 memory report
  void report_memory() {
    long v[3] = {(long)(buffsize * sizeof(T)), (long)(recycle * sizeof(T)), (long)(reuse * sizeof(T))};
    MPI_Allreduce(MPI_IN_PLACE, v, 3, MPI_LONG, MPI_SUM, CommBench::comm_mpi);
    if (CommBench::myid == CommBench::printid) {
      std::printf("total buffsize: ");
      CommBench::print_data(v[0]);
      std::printf(" reuse: ");
      CommBench::print_data(v[2]);
      std::printf(" recycle: ");
      CommBench::print_data(v[1]);
      std::printf("\n");
    }
  }
};

}  // namespace HiCCL

#endif  // HICCL_COMM_H
