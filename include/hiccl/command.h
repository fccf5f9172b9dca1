// include/hiccl/command.h -- lowering of the per-batch level lists into the
// executable pipeline (reference: source/command.h).
//
//   merge_steps   command.h:84-156 semantics: batch b starts b*pipeoffset
//                 steps late (the reference pushes dummy colls, 89-90); at
//                 every step the colls of all batches are merged per library;
//                 steps without work are dropped.
//   Command       one (transport, compute) pair per library per step
//                 (command.h:2-38), measure() as command.h:17-37.
//   instantiate   builds the transports and the computes of every step; on
//                 the MI355X port each step's Compute is ONE batched kernel.
#ifndef HICCL_COMMAND_H
#define HICCL_COMMAND_H

#include <list>
#include <vector>

#include "compute.h"
#include "plan.h"

namespace HiCCL {

// Libraries used by any level of any batch, in enum order (command.h:76-92).
template <typename T>
std::vector<CommBench::library> libraries_used(const std::vector<CollList<T>> &batches) {
  std::vector<bool> used(CommBench::numlib, false);
  for (auto &b : batches)
    for (auto *c : b) used[c->lib] = true;
  std::vector<CommBench::library> libs;
  for (int l = 0; l < CommBench::numlib; l++)
    if (used[l]) libs.push_back((CommBench::library)l);
  return libs;
}

// steps[s][i] = everything library libs[i] does at step s.
template <typename T>
std::vector<std::vector<Coll<T>>> merge_steps(const std::vector<CollList<T>> &batches,
                                              const std::vector<CommBench::library> &libs, int pipeoffset) {
  std::vector<int> slot(CommBench::numlib, -1);
  for (size_t i = 0; i < libs.size(); i++) slot[libs[i]] = (int)i;
  std::vector<std::vector<const Coll<T> *>> lanes(batches.size());
  size_t depth = 0;
  for (size_t b = 0; b < batches.size(); b++) {
    lanes[b].assign(b * pipeoffset, nullptr);  // stagger
    for (auto *c : batches[b]) lanes[b].push_back(c);
    depth = std::max(depth, lanes[b].size());
  }
  std::vector<std::vector<Coll<T>>> steps;
  for (size_t s = 0; s < depth; s++) {
    std::vector<Coll<T>> step;
    for (auto l : libs) step.emplace_back(l);
    bool work = false;
    for (auto &lane : lanes) {
      if (s >= lane.size() || !lane[s]) continue;
      const Coll<T> &c = *lane[s];
      Coll<T> &dst = step[slot[c.lib]];
      dst.xfers.insert(dst.xfers.end(), c.xfers.begin(), c.xfers.end());
      dst.comps.insert(dst.comps.end(), c.comps.begin(), c.comps.end());
      work = work || !c.empty();
    }
    if (work) steps.push_back(std::move(step));
  }
  return steps;
}

template <typename T>
struct Command {
  CommBench::Comm<T> *comm = nullptr;
  Compute<T> *compute = nullptr;

  Command(CommBench::Comm<T> *c, Compute<T> *k) : comm(c), compute(k) {}

  // command.h:17-37: time the transport, then (if any rank computes) the
  // compute stage, each on its own.
  void measure(int warmup, int numiter, size_t count) {
    int ncomm = comm->numsend + comm->numrecv, ncomp = compute->numcomp;
    MPI_Allreduce(MPI_IN_PLACE, &ncomm, 1, MPI_INT, MPI_SUM, CommBench::comm_mpi);
    MPI_Allreduce(MPI_IN_PLACE, &ncomp, 1, MPI_INT, MPI_SUM, CommBench::comm_mpi);
    if (CommBench::myid == CommBench::printid)
      std::printf("COMMAND TYPE: %s\n", ncomm ? (ncomp ? "COMMUNICATION + COMPUTATION" : "COMMUNICATION")
                                              : (ncomp ? "COMPUTATION" : "NONE"));
    if (ncomm) comm->measure(warmup, numiter, count);
    if (ncomp) compute->measure(warmup, numiter, count);
  }
};

// Build every step's transports and computes.  pipeline[i] is library i's
// list of commands, one per step (the reference's command_batch).
// `fuse`: transfers whose receive buffer only feeds a compute of the same
// step (Coll::Xfer::feeds) are not copied; the compute reads the sender's
// buffer in place through its IPC mapping (fused gather + reduce).
template <typename T>
std::vector<std::list<Command<T>>> instantiate(const std::vector<std::vector<Coll<T>>> &steps,
                                               const std::vector<CommBench::library> &libs, bool fuse = false) {
  std::vector<std::list<Command<T>>> pipeline(libs.size());
  for (auto &step : steps) {
    for (size_t i = 0; i < libs.size(); i++) {
      auto *comm = new CommBench::Comm<T>(libs[i]);
      auto *comp = new Compute<T>();
      for (auto &x : step[i].xfers)
        comm->add(x.sendbuf, x.sendoffset, x.recvbuf, x.recvoffset, x.count, x.sendid, x.recvid, fuse && x.feeds);
      for (auto &c : step[i].comps) {
        std::vector<T *> in = c.inputs;
        bool peer = false;  // an input read in place from a peer's buffer
        if (fuse && c.compid == CommBench::myid)
          for (auto &p : in)
            if (T *remote = comm->fused_source(p)) {
              p = remote;
              peer = true;
            }
        comp->add(in, c.output, c.count, c.compid, peer);
      }
      pipeline[i].emplace_back(comm, comp);
    }
  }
  return pipeline;
}

}  // namespace HiCCL

#endif  // HICCL_COMMAND_H
