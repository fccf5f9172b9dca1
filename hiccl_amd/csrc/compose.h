// hiccl_amd/csrc/compose.h -- the eight collective compositions of the
// reference driver (collectives/main.cpp:104-160), written against any
// "sink" with fence() / reduce(...) / bcast(...) so the same composition
// feeds HiCCL::Comm<T> (the driver) and HiCCL::Schedule<T> (plan dumps).
#ifndef HICCL_COMPOSE_H
#define HICCL_COMPOSE_H

#include <vector>

#include "../../include/hiccl.h"

namespace hiccl_driver {

inline std::vector<int> ids(int id, int np, int other) { return HiCCL::expand_ids(id, np, other); }

// Pattern ids as hiccl.h:41 (enum collective).
template <typename Sink, typename T>
bool compose(Sink &s, int pattern, T *sendbuf, T *recvbuf, size_t count, int np, int root) {
  using namespace HiCCL;
  switch (pattern) {
    case gather:
      for (int p = 0; p < np; p++) s.bcast(sendbuf, 0, recvbuf, p * count, count, p, ids(root, np, p));
      return true;
    case scatter:
      for (int p = 0; p < np; p++) s.reduce(sendbuf, p * count, recvbuf, 0, count, ids(root, np, p), p);
      return true;
    case broadcast:
      s.bcast(sendbuf, 0, recvbuf, 0, count * np, root, ids(np, np, root));
      return true;
    case reduce:
      s.reduce(sendbuf, 0, recvbuf, 0, count * np, ids(np, np, root), root);
      return true;
    case alltoall:
      for (int p = 0; p < np; p++)
        for (int q = 0; q < np; q++) s.bcast(sendbuf, q * count, recvbuf, p * count, count, p, ids(q, np, p));
      return true;
    case allgather:
      for (int p = 0; p < np; p++) s.bcast(sendbuf, 0, recvbuf, p * count, count, p, ids(np, np, p));
      return true;
    case reducescatter:
      for (int p = 0; p < np; p++) s.reduce(sendbuf, p * count, recvbuf, 0, count, ids(np, np, p), p);
      return true;
    case allreduce:  // reduce-scatter + fence + all-gather (collectives/main.cpp:151-155)
      for (int p = 0; p < np; p++) s.reduce(sendbuf, p * count, recvbuf, p * count, count, ids(np, np, p), p);
      s.fence();
      for (int p = 0; p < np; p++) s.bcast(recvbuf, p * count, recvbuf, p * count, count, p, ids(-1, np, p));
      return true;
    default:
      return false;
  }
}

// Adapter: Comm<T>'s public API as a sink.
template <typename T>
struct CommSink {
  HiCCL::Comm<T> &c;
  void fence() { c.add_fence(); }
  void reduce(T *sb, size_t so, T *rb, size_t ro, size_t n, std::vector<int> ids, int rid) {
    c.add_reduce(sb, so, rb, ro, n, ids, rid);
  }
  void bcast(T *sb, size_t so, T *rb, size_t ro, size_t n, int sid, std::vector<int> ids) {
    c.add_bcast(sb, so, rb, ro, n, sid, ids);
  }
};

}  // namespace hiccl_driver

#endif
