/*
 * hiccl_reduce.h -- C ABI of the MI355X (gfx950) bucket-reduction stage.
 *
 * This is the drop-in boundary for HiCCL's local reduction compute stage:
 * element-wise, in-order sum of N gathered device buffers into one output,
 *
 *     out[i] = ((((T)0 + in[0][i]) + in[1][i]) + ...) + in[n-1][i]
 *
 * with every add rounded to T (reference: source/compute.h:2-12 GPU
 * reduce_kernel<T>, compute.h:14-23 CPU reduce_kernel<T>).  Results are
 * bit-identical to the reference's reduction on the same inputs.
 *
 * Plain C: pointers, sizes and ints only.  `stream` is a hipStream_t passed
 * as void* (NULL = the default stream), device pointers are plain void*.
 * Every function returns a hipError_t value as int (0 = hipSuccess); invalid
 * arguments return hipErrorInvalidValue (1) and leave a message readable with
 * hiccl_last_error().
 *
 * Implementation: hiccl_amd/csrc/reduce.hip -> hiccl_amd/libhiccl_reduce.so
 * Design and roofline: DESIGN.md.  Reference-side bindings: INTEGRATION.md.
 */
#ifndef HICCL_REDUCE_H
#define HICCL_REDUCE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Element types.  The reference is a template over T (compute.h:26); its
 * drivers instantiate T = size_t (collectives/main.cpp:24, main.cpp:4) and
 * T = float (main.cu:10).  bf16 follows `T acc; acc += x` semantics
 * (round to bf16 after every add) unless HICCL_ACC_WIDE is requested. */
typedef enum {
  HICCL_FLOAT32 = 0,
  HICCL_FLOAT64 = 1,
  HICCL_BFLOAT16 = 2,
  HICCL_UINT64 = 3, /* size_t */
  HICCL_INT32 = 4,
  HICCL_BYTES = 5,  /* exact copy, exactly one input: out = in[0] (transport data movement) */
  HICCL_NUM_DTYPES = 6
} hiccl_dtype_t;

/* Accumulation mode (only meaningful for HICCL_BFLOAT16). */
typedef enum {
  HICCL_ACC_NATIVE = 0, /* accumulate in T: reference semantics (default) */
  HICCL_ACC_WIDE = 1    /* accumulate bf16 in f32, round once: NOT reference-bitwise */
} hiccl_acc_t;

/* Kernel engine (both compute the same bits; they differ in access order).
 *   TILE   all n inputs of a 16 KiB-per-input tile are loaded together.
 *   PHASE  a workgroup sweeps a 128 KiB chunk of input 0, then of input 1,
 *          ... (next input's loads in flight while the current one is
 *          added), then writes the chunk.
 *   AUTO   TILE (on the dynamic schedule, below) with >= 5 inputs once
 *          every workgroup gets >= 64 tickets (bf16: packed accumulator
 *          only); TILE with 32 KiB-per-input tiles (unroll 8) on the
 *          dynamic schedule with 2-4 inputs once every workgroup gets
 *          >= 128 of them (1 GiB per input, f32 / bf16); otherwise PHASE
 *          when its chunks fill the CUs: >= 1 chunk per CU with >= 5
 *          inputs (with >= 16 inputs and 128 KiB chunks 0.7 suffice), >= 4
 *          with 3-4, > 16 with 2, in rounds of chunks that keep >= 70 % (64
 *          KiB chunks: 80 %) / ~90 % / ~90 % of the CUs busy -- else TILE,
 *          with 4 workgroups per CU below one chunk per CU (unroll 2 below
 *          two 16 KiB tiles per CU) (one-shot: that call; plan: all
 *          computes, packet-weighted mean n). */
typedef enum {
  HICCL_ENGINE_AUTO = 0,
  HICCL_ENGINE_TILE = 1,
  HICCL_ENGINE_PHASE = 2
} hiccl_engine_t;

/* Work-unit schedule (same bits either way).
 *   STATIC   workgroup b takes units b, b + grid, ...
 *   DYNAMIC  workgroups take their next `grab` units from a device counter
 *            (one per device and stream, reset by the launch itself):
 *            faster-served workgroups do more units, the tail is one ticket.
 *   AUTO     DYNAMIC for the TILE engine with >= 5 inputs and >= 32 tickets
 *            per workgroup, STATIC otherwise.
 * Always STATIC during stream capture (a replayed graph must not share a
 * stream's counter) and on hipStreamPerThread (one handle value, a different
 * stream per host thread).  A forced DYNAMIC still needs >= 32 tickets per
 * workgroup.  Plans take the schedule of hiccl_reduce_plan_set_config
 * (default AUTO). */
typedef enum {
  HICCL_SCHED_AUTO = 0,
  HICCL_SCHED_STATIC = 1,
  HICCL_SCHED_DYNAMIC = 2
} hiccl_schedule_t;

/* Size in bytes of one element of `dtype`, 0 if unknown. */
size_t hiccl_dtype_size(int dtype);

/* Message describing the last error returned on this host thread. */
const char *hiccl_last_error(void);

/* Library version as MAJOR*10000 + MINOR*100 + PATCH. */
int hiccl_version(void);

/* ----------------------------------------------------------------------
 * One-shot reduction.  Replaces one registered compute of the reference's
 * Compute<T> being launched: compute.h:90-91 (launch of reduce_kernel with
 * the device pointer table built at compute.h:70-72).
 *
 *   in     HOST array of n DEVICE pointers, in summation order (the order
 *          reduce.h:134-169 emits: ascending rank).  Copied at call time;
 *          the caller may free it on return.
 *   out    device pointer; may equal one of the inputs exactly (in-place);
 *          partial overlap with an input is not allowed.
 *   count  elements; 0 is a no-op.  n == 0 writes T(0) to every element.
 *   Pointers need only be element-aligned; inputs may be mutually
 *   misaligned (element offsets from reduce.h:401-415 partition()).
 *   Asynchronous on `stream`.
 */
int hiccl_reduce(int dtype, void *out, const void *const *in, int n, size_t count,
                 void *stream);
int hiccl_reduce_f32(float *out, const float *const *in, int n, size_t count, void *stream);
int hiccl_reduce_bf16(uint16_t *out, const uint16_t *const *in, int n, size_t count,
                      void *stream);

/* Tuning knobs of the single-compute kernel.  Zero fields mean "default".
 * With engine AUTO, a non-zero block or unroll selects the TILE engine.
 * With n > 64 inputs the call runs on the plan kernel (pointer table in
 * device memory), which has fewer shapes (hiccl_reduce_plan_set_config): a
 * shape it lacks is an error, never silently replaced; such a call cannot
 * be captured into a graph (hipErrorStreamCaptureUnsupported). */
typedef struct {
  int block;         /* threads per workgroup: TILE 256 or 512; PHASE 256, 512 or 1024 */
  int unroll;        /* 16-byte packets per input per lane per tile: TILE 1, 2 or 4 (block
                        256, f32 / bf16: also 8 or 16 -- wide tiles for few inputs);
                        PHASE 4, 8 or 16 (chunk = block * unroll * 16 B) */
  int blocks_per_cu; /* persistent grid = CUs x this (capped by tiles) */
  int nontemporal;   /* loads: 1 plain cache policy, 2 nt */
  int acc;           /* hiccl_acc_t */
  int grid;          /* total workgroups; overrides blocks_per_cu when > 0 */
  int store_policy;  /* stores: 1 plain, 2 nt, 3 sc1 (write-through, line dropped from L2),
                        4 system-scope write-through (sc0 sc1).  0: 4 when the launch
                        writes at most 256 MiB of sums (two or more inputs) or 32 MiB
                        of copies (one input), its loads are nt and its shape has a
                        write-through kernel -- no dirty L2 lines left for the kernel
                        boundary -- else 2.  The shapes the size rule applies to,
                        one-shot calls and plans alike: AUTO, TILE unroll 2 / 4,
                        PHASE's default shape (an explicit TILE unroll 1, 8 or 16
                        stays nt; one-shot unroll 1 stores write-through on
                        request, 4).  The store form is decided before AUTO picks
                        the engine (its rules differ under write-through) */
  int engine;        /* hiccl_engine_t */
  int schedule;      /* hiccl_schedule_t */
  int grab;          /* dynamic schedule: units per ticket (0 = default: PHASE 1,
                        TILE ceil(9 / (n + 1))) */
  int drain;         /* 1: a workgroup waits for a unit's stores before the next unit's loads */
  int order;         /* one-shot calls (n <= 64): units run interleaved over `order` equal
                        stretches of the bucket (a power of two <= 4096; 0 / 1: linear);
                        plans: 0 only */
} hiccl_reduce_config_t;

int hiccl_reduce_ex(int dtype, void *out, const void *const *in, int n, size_t count,
                    void *stream, const hiccl_reduce_config_t *cfg);

/* What AUTO (engine, TILE unroll / PHASE packets per lane, workgroups per
 * CU, dynamic unit schedule 1/0) picks for a one-shot call of n inputs of
 * `count` elements whose output is 16-B aligned and whose store form is left
 * to size (store_policy 0), on a GPU of `cus` CUs (no
 * device is queried: host code and tests can ask; a plan asks with the sum
 * of its computes' elements and their packet-weighted mean n).  A launch on
 * a capturing stream or hipStreamPerThread takes the static schedule. */
int hiccl_reduce_auto_choice(int dtype, int acc, size_t count, double n, int cus, int *engine, int *unroll,
                             int *blocks_per_cu, int *dynamic);
/* The same for a one-shot call with config `cfg` (NULL = defaults), the same
 * resolution hiccl_reduce_ex makes -- store form first, then engine and
 * shape -- plus the store form it takes (*store_policy: 2 nt, 4
 * write-through; any pointer may be NULL).  A config no kernel has returns
 * hipErrorInvalidValue, as hiccl_reduce_ex would.  A plan of one compute
 * with TILE unroll 2 / 4 or AUTO resolves the same way (tests pin the GPU
 * tier's AUTO expectations to this answer on the host). */
int hiccl_reduce_auto_choice_ex(int dtype, const hiccl_reduce_config_t *cfg, size_t count, double n, int cus,
                                int *engine, int *unroll, int *blocks_per_cu, int *dynamic, int *store_policy);

/* ----------------------------------------------------------------------
 * Persistent plan: the C-ABI counterpart of the reference's Compute<T>
 * (compute.h:26-204).  A plan holds any number of registered computes and
 * launches ALL of them in ONE kernel (one launch per pipeline step instead
 * of one launch + one stream per compute, compute.h:87-106).
 *
 *   create   compute.h:26-45 (object) -- binds `device`.
 *   add      compute.h:47-85 add(inputbuf, outputbuf, count, compid):
 *            records one compute; `in` is a HOST array of n DEVICE
 *            pointers, copied.  (The reference's SPMD "only if myid ==
 *            compid" filter, compute.h:66, is applied by the C++ caller.)
 *   launch   compute.h:87-106 start(): one batched kernel on `stream`
 *            (NULL = the default stream, as everywhere in this ABI; the
 *            plan's own stream -- the reference creates one per compute,
 *            compute.h:76-78 -- is hiccl_reduce_plan_stream()).  The first
 *            launch after an add or a config change uploads the descriptor
 *            table (synchronous, once; refused inside a stream capture).
 *   sync     compute.h:107-117 wait(): hipStreamSynchronize of the stream
 *            of the plan's last launch (as the reference synchronises each
 *            compute's stream) -- that stream must still exist.  No event is
 *            recorded per launch.
 *   destroy  frees the plan's device tables and stream (the reference leaks
 *            them, compute.h:70-82).
 * Threading: launch/sync may be called from a different host thread than
 * create/add (Comm::start's pthread, comm.h:214-224); each entry binds the
 * plan's device.  Not reentrant per plan; distinct plans are independent.
 */
typedef struct hiccl_reduce_plan hiccl_reduce_plan_t;

int hiccl_reduce_plan_create(hiccl_reduce_plan_t **plan, int dtype, int device);
int hiccl_reduce_plan_set_acc(hiccl_reduce_plan_t *plan, int acc);
/* Engine for the plan's launches (hiccl_engine_t; default AUTO, decided from
 * the total packets of all computes at the first launch after an add). */
int hiccl_reduce_plan_set_engine(hiccl_reduce_plan_t *plan, int engine);
/* Kernel configuration of the plan's launches (NULL = all defaults; replaces
 * earlier set_engine / set_acc choices).  Honoured: engine, schedule, grab,
 * blocks_per_cu, grid, acc, and the TILE shape block 256 x unroll 4 (f32 and
 * bf16 also unroll 1, 2, 8 or 16); PHASE runs its default shape; loads are
 * nt; stores are nt (store_policy 2), system-scope write-through (4), or
 * (0, the default) write-through when a launch writes at most 256 MiB of
 * sums or 32 MiB of byte copies and nt above -- pipeline steps and mid-size
 * buckets, where nt lines left dirty in the L2s cost the kernel boundary
 * their write-back -- except
 * for an explicit TILE unroll 1, 8 or 16, which stays nt.  Write-through
 * runs the shapes the peer kernels have (below).  Anything else is refused
 * with hipErrorInvalidValue -- no field is silently ignored. */
int hiccl_reduce_plan_set_config(hiccl_reduce_plan_t *plan, const hiccl_reduce_config_t *cfg);
/* Peer memory.  The transport's data movement (the CommBench IPC put / get
 * the reference registers at command.h:122,132 and starts at comm.h:190,197)
 * and the fused gather + reduce (reduce.h:134-170's receive buffers read in
 * place) run plans whose outputs or inputs live in ANOTHER GPU's memory
 * (HIP IPC mappings over xGMI).  Their launches must hand bytes to, or take
 * them from, a kernel of the other GPU in the same stream-ordered pipeline,
 * with only a device-side flag in between:
 *   HICCL_PEER_STORES  every store is system-scope write-through (nothing of
 *                      a peer's buffer stays dirty in this GPU's L2s after
 *                      the kernel);
 *   HICCL_PEER_LOADS   every load is system-scope coherent (no L2 line of a
 *                      peer's buffer cached by an earlier launch is served).
 * Same results; runs the PHASE engine's default shape and TILE at unroll 4
 * (f32 / bf16 also 2): an automatic wide-tile choice becomes unroll 4, an
 * explicit unroll the peer kernels lack fails at launch.  Kept by
 * hiccl_program_add_plan for the plan's computes. */
typedef enum {
  HICCL_PEER_STORES = 1,
  HICCL_PEER_LOADS = 2
} hiccl_peer_t;
int hiccl_reduce_plan_set_peer(hiccl_reduce_plan_t *plan, int flags);
/* The plan's peer flags (-1 for NULL). */
int hiccl_reduce_plan_peer(const hiccl_reduce_plan_t *plan);
/* The store form the plan's launches take with its current computes and
 * config (hiccl_reduce_config_t.store_policy: 2 nt, 4 system-scope
 * write-through; -1 for NULL). */
int hiccl_reduce_plan_store_policy(const hiccl_reduce_plan_t *plan);
/* The engine the last upload resolved to (TILE before the first launch). */
int hiccl_reduce_plan_engine(const hiccl_reduce_plan_t *plan);
int hiccl_reduce_plan_add(hiccl_reduce_plan_t *plan, void *out, const void *const *in, int n,
                          size_t count);
int hiccl_reduce_plan_launch(hiccl_reduce_plan_t *plan, void *stream);
/* launch without remembering the stream for hiccl_reduce_plan_sync: for
 * stream-ordered callers that synchronise the stream themselves, and for
 * launches from several threads onto different streams.  A later re-upload
 * (the first launch after an add or a config change) or destroy of a plan
 * launched this way synchronises the device before it frees the plan's
 * device table. */
int hiccl_reduce_plan_enqueue(hiccl_reduce_plan_t *plan, void *stream);
/* Reference structure, for measurement: one kernel per compute, each on
 * the given stream (compute.h:88-91 launches one kernel per compute) --
 * each one a one-shot hiccl_reduce_ex with the plan's configuration (AUTO
 * decides per compute). */
int hiccl_reduce_plan_launch_each(hiccl_reduce_plan_t *plan, void *stream);
/* Waits for the last hiccl_reduce_plan_launch (hipStreamSynchronize of its
 * stream, compute.h:107-117).  After it returns the plan no longer refers to
 * that stream: the caller may destroy the stream.  A plan destroyed or
 * re-uploaded while a launch was never synchronised synchronises the launch's
 * stream, which must then still exist. */
int hiccl_reduce_plan_sync(hiccl_reduce_plan_t *plan);
/* The plan's own non-blocking stream (a hipStream_t), created on the first
 * call and destroyed with the plan; NULL on error. */
void *hiccl_reduce_plan_stream(hiccl_reduce_plan_t *plan);
int hiccl_reduce_plan_numcomp(const hiccl_reduce_plan_t *plan);
/* Sum over computes of count * (n + 1) * sizeof(T): the bytes the reference's
 * measure(warmup, numiter) overload (compute.h:197-203) prices. */
size_t hiccl_reduce_plan_bytes(const hiccl_reduce_plan_t *plan);
void hiccl_reduce_plan_destroy(hiccl_reduce_plan_t *plan);

/* ----------------------------------------------------------------------
 * Host-resident buckets.
 *
 * The reference reduces host arrays with its host port (reduce_kernel,
 * compute.h:14-23) and stages host<->device copies around the device path
 * in its benchmarks (bench.h:80-108).  A host pipe reduces n host-resident
 * inputs into a host-resident output on the GPU: the bucket is cut into
 * chunks of chunk_bytes per input; chunk c's n H2D copies, its reduction
 * (hiccl_reduce, in place into the staged input 0) and its D2H copy run on
 * stream c % depth, so the two PCIe directions and the kernel overlap.
 * Same bits as hiccl_reduce on the same inputs.  Pinned memory
 * (hipHostMalloc / hipHostRegister) is needed for the overlap; pageable
 * memory gives the same result with serialised copies.
 *   create   chunk_bytes 0 = 64 MiB per input; depth 0 = 3 (1..8 allowed);
 *            device staging (depth x n x chunk_bytes) is allocated on the
 *            first reduce and grows with n.
 *   reduce   blocking: returns when out holds the sum.  Pointers must be
 *            element-aligned; partial overlaps are refused.
 *   destroy  frees staging and streams.
 */
typedef struct hiccl_host_pipe hiccl_host_pipe_t;

int hiccl_host_pipe_create(hiccl_host_pipe_t **pipe, int dtype, int device, size_t chunk_bytes,
                           int depth);
int hiccl_host_pipe_reduce(hiccl_host_pipe_t *pipe, void *out, const void *const *in, int n,
                           size_t count);
void hiccl_host_pipe_destroy(hiccl_host_pipe_t *pipe);

/* ----------------------------------------------------------------------
 * Stream-ordered signalling for the transport (include/hiccl/transport.h).
 *
 * Enqueues on `stream` (after all earlier work on it): a system-scope store
 * of `epoch` to each of the nsig flags `sig` (typically flags in a peer's
 * IPC-mapped device memory), then a bounded spin until each of the nwait
 * local flags `wait` holds a value >= epoch (32-bit wrap-aware).  The
 * stores are system-scope releases and the polls acquires
 * (hiccl_token_mode; HICCL_PROG_FENCES=light makes both relaxed).  A token
 * orders launches; data it announces must be complete when the launch that
 * wrote it ended -- written through to a peer's memory with
 * hiccl_reduce_plan_set_peer.  A spin exceeding timeout_s (<= 0: 30 s) stores
 * 1 to *err (if err is not NULL; host-visible memory recommended) and gives
 * up instead of hanging.  Replaces, per pipeline step, the host round trip
 * the reference's transport makes around every transfer (comm.h:188-204).
 */
int hiccl_signal_wait(uint32_t *const *sig, int nsig, const uint32_t *const *wait, int nwait,
                      uint32_t epoch, uint32_t *err, double timeout_s, void *stream);
/* Graph-replayable form: the epoch used is epoch + *epoch_dev, read when the
 * wait runs (epoch_dev NULL: epoch alone), so a captured hipGraph advances
 * its epochs through a device counter bumped once per replay with
 * hiccl_counter_add (one lane, stream-ordered: *ctr += v). */
int hiccl_signal_wait_dev(uint32_t *const *sig, int nsig, const uint32_t *const *wait, int nwait,
                          uint32_t epoch, const uint32_t *epoch_dev, uint32_t *err, double timeout_s,
                          void *stream);
int hiccl_counter_add(uint32_t *ctr, uint32_t v, void *stream);
/* Several signal/wait steps in order, in as few launches as possible (one
 * 64-lane wave runs up to 8 phases, 64 signal and 64 wait flags): phase p
 * signals its flags with its epoch, then waits for its flags; phase p + 1
 * starts after every wait of phase p.  Same effect as one
 * hiccl_signal_wait_dev per phase, with fewer kernel boundaries on the
 * stream (the transport merges a step's done tokens with the next step's
 * readies this way).  A phase with more than 64 flags of a kind signals all
 * of them before its first wait. */
typedef struct {
  uint32_t *const *sig;
  int nsig;
  const uint32_t *const *wait;
  int nwait;
  uint32_t epoch;
} hiccl_signal_phase_t;
int hiccl_signal_wait_phases(const hiccl_signal_phase_t *phases, int nphases, const uint32_t *epoch_dev,
                             uint32_t *err, double timeout_s, void *stream);

/* ----------------------------------------------------------------------
 * Programs: token phases folded into the kernel of the work they guard
 * (stream-ordered transport).
 *
 * The reference runs a step as transport start -> transport wait -> compute
 * start -> compute wait (comm.h:195-204); the stream-ordered port enqueues a
 * hiccl_signal_wait_phases before every copy and reduction kernel.  A
 * program is ONE launch of: the phases (run first, in order, by one wave,
 * as hiccl_signal_wait_phases does), then the units of one batch of
 * computes -- plans' computes, reductions of the program's dtype or
 * HICCL_BYTES exact copies, all independent of each other -- which start
 * only after the last phase.  Same stores, waits and results as the
 * separate launches (the same token mode), one kernel boundary fewer
 * per phase group.
 *
 * add_signal appends one phase (only before the first add_plan); its epoch
 *   is supplied per launch.
 * add_plan appends the plan's computes as of this call (later adds to the
 *   plan are not seen); the plan's dtype must be the program's or
 *   HICCL_BYTES; native accumulation only.  Computes of several plans form
 *   one batch: they must not depend on each other.  Each plan's store form
 *   carries over as the plan decided it (hiccl_reduce_plan_store_policy, by
 *   that plan's own size): a program joining several plans may write more
 *   than the 256 MiB / 32 MiB caps in one launch and still store
 *   write-through (a pipeline step's batches are a few MiB).
 * launch: epochs[p] for every phase p (+ *epoch_dev when not NULL, read at
 *   run time: graph replays), err / timeout_s as hiccl_signal_wait.  The
 *   first launch (and the first after a change) uploads the program's tables
 *   and cannot be captured into a graph.  One launch of a program at a time
 *   (launches on one stream).
 * Limit: 64 phases per program.
 */
typedef struct hiccl_program hiccl_program_t;
int hiccl_program_create(hiccl_program_t **prog, int dtype, int device);
int hiccl_program_add_signal(hiccl_program_t *prog, uint32_t *const *sig, int nsig, const uint32_t *const *wait,
                             int nwait);
int hiccl_program_add_plan(hiccl_program_t *prog, const hiccl_reduce_plan_t *plan);
/* Cap the launch at max_wg workgroups (0: the default, 2-4 per CU).
 * Processes sharing one GPU (rehearsals) split it this way: a program's
 * workgroups wait on the GPU for its phases, i.e. for peers' tokens. */
int hiccl_program_set_max_workgroups(hiccl_program_t *prog, int max_wg);
int hiccl_program_num_units(const hiccl_program_t *prog);
int hiccl_program_num_phases(const hiccl_program_t *prog);
int hiccl_program_launch(hiccl_program_t *prog, const uint32_t *epochs, const uint32_t *epoch_dev, uint32_t *err,
                         double timeout_s, void *stream);
void hiccl_program_destroy(hiccl_program_t *prog);

/* Stream-ordered protocol defaults, resolved from the environment at each
 * call (launches resolve them the same way; no device needed).
 *   hiccl_token_mode: the token phases of hiccl_signal_wait* and programs.
 *     HICCL_TOKENS_FENCED (default; HICCL_PROG_FENCES unset, "full" or any
 *     other value): system-scope release token stores, relaxed polls closed
 *     by a system-scope acquire fence per phase (the fence form of an
 *     acquire load), a release gate store, and in a program's other
 *     workgroups an agent-scope acquire fence after their gate polls --
 *     every token and the gate hand-off ordered by the memory model.
 *     HICCL_TOKENS_LIGHT (HICCL_PROG_FENCES=light): relaxed stores and
 *     polls, no fences; the same cost for per-element launches, cheaper for
 *     programs on one GPU, but its argument (tokens
 *     publish nothing of their own launch) leans on kernel-boundary cache
 *     behaviour across GPUs that no run with one GPU per rank has confirmed
 *     yet, so it is opt-in.
 *   hiccl_step_program_default: 1 when HiCCL::Comm's stream-ordered mode folds
 *     token phases into step programs (HICCL_STEP_PROGRAM=1, yes, on or true,
 *     any case), else 0 -- one launch per element, the protocol the GPU
 *     suite verifies by default; an unrecognised value reads as 0 and is
 *     named once on stderr. */
#define HICCL_TOKENS_FENCED 0
#define HICCL_TOKENS_LIGHT 1
int hiccl_token_mode(void);
int hiccl_step_program_default(void);

/* ----------------------------------------------------------------------
 * Measurement utilities (bench.py; not part of the reference surface).
 *
 * fill_uniform: element i of buffer k = uniform [-1,1) value of hash
 * (seed, k, first + i), identical to oracle/reduce_oracle.c's generator
 * (dtypes FLOAT32, BFLOAT16, FLOAT64).
 * stream_copy: plain 16-byte-per-lane device copy, the achievable-bandwidth
 * ceiling reference for the roofline.
 */
int hiccl_fill_uniform(int dtype, void *out, size_t count, uint64_t seed, uint32_t k,
                       size_t first, void *stream);
int hiccl_stream_copy(void *dst, const void *src, size_t bytes, void *stream);
/* hipDeviceProp values the roofline is checked against: CUs, peak memory
 * clock (kHz) and memory bus width (bits); NULL outputs are skipped. */
int hiccl_device_info(int device, int *cus, int *mem_clock_khz, int *bus_width_bits);

/* ----------------------------------------------------------------------
 * Bucket layout.  A reduction bucket -- n inputs and the output of one
 * compute, `count` elements each -- in ONE device allocation: buffer j
 * (inputs 0..n-1, then the output) at base + j * hiccl_bucket_stride(dtype,
 * count), the buffer's bytes rounded up to 64 KiB plus 64 KiB.  Separate
 * allocations leave the relative physical placement of the n + 1 streams to
 * chance, and config 2's kernel time moves by up to 8 % with it; buckets in
 * one allocation run at the fast end, every instance.
 * The reduction reads and writes exactly the same bytes either way.
 *   stride   bytes between consecutive buffers (0 for an unknown dtype or
 *            count 0).
 *   alloc    hipMalloc on `device` of (n + 1) strides; in[k] (a host array
 *            of n pointers) and *out receive the buffers, *base the
 *            allocation to pass to hiccl_bucket_free.
 */
size_t hiccl_bucket_stride(int dtype, size_t count);
int hiccl_bucket_alloc(int dtype, int n, size_t count, int device, void **base, void **in, void **out);
int hiccl_bucket_free(void *base);

#ifdef __cplusplus
}
#endif

#endif /* HICCL_REDUCE_H */
