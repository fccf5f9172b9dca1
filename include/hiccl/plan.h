// include/hiccl/plan.h -- HiCCL primitives and their factorization into
// per-level transfer/compute sets (the IR).
//
// The factorization decides every compute's input list, input ORDER, element
// count and offsets, i.e. the summation order of the result, so it follows
// the reference exactly (checked against oracle/schedule.py, which restates
// the reference, and against the compiled-reference probe of SURVEY.md 8c):
//
//   REDUCE / BROADCAST pattern expansion   reduce.h:51-66, broadcast.h:52-66
//   reduce tree (innermost level first)    reduce.h:69-211
//   reduce ring                            reduce.h:213-335
//   striping                               reduce.h:337-399, broadcast.h:238-319
//   pipelining split                       reduce.h:401-415, broadcast.h:321-335
//   broadcast tree / ring                  broadcast.h:69-172, 174-236
//
// Design differences (same results):
//   * a Planner object carries the rank context (me, numproc) and the
//     allocator, so the whole factorization can be run for every rank of a
//     virtual machine in one process (tests/cpp/plan_dump.cpp);
//   * pointers that only exist on another rank are nullptr, not garbage;
//   * pooled receive buffers remember their capacity (the reference reuses a
//     recycled buffer whatever the new count, reduce.h:139-145);
//   * ring forwarding never reduces into a user send buffer: the reference
//     reuses the next node's send buffer as the ring partial whenever that
//     node's only sender is the forwarding rank (reduce.h:261-270), even when
//     further nodes still have to be reduced into it, which overwrites the
//     user's send buffer and drops that rank's contribution (only reachable
//     with one rank per ring node).  Here the buffer is reused only when the
//     rest of the ring is empty (the case where the reference is correct).
#ifndef HICCL_PLAN_H
#define HICCL_PLAN_H

#include <cstdio>
#include <algorithm>
#include <functional>
#include <list>
#include <utility>
#include <vector>

#include "transport.h"

namespace HiCCL {

// reduce.h:54-66 / broadcast.h:54-66: an id of numproc means every rank,
// -1 every rank but `other`, anything else that single rank.
inline std::vector<int> expand_ids(int id, int np, int other) {
  std::vector<int> v;
  for (int i = 0; i < np; i++)
    if (id == np || (id == -1 && i != other) || i == id) v.push_back(i);
  return v;
}

template <typename T>
inline T *at(T *p, size_t off) {
  return p ? p + off : nullptr;
}

// Reduction primitive (reduce.h:2-67): sendbuf/sendoffset are rank-local.
template <typename T>
struct REDUCE {
  T *sendbuf;
  size_t sendoffset;
  T *recvbuf;
  size_t recvoffset;
  size_t count;
  std::vector<int> sendids;
  int recvid;
  REDUCE(T *sb, size_t so, T *rb, size_t ro, size_t c, std::vector<int> ids, int rid)
      : sendbuf(sb), sendoffset(so), recvbuf(rb), recvoffset(ro), count(c), sendids(std::move(ids)), recvid(rid) {}
};

// Multicast primitive (broadcast.h:2-67).
template <typename T>
struct BROADCAST {
  T *sendbuf;
  size_t sendoffset;
  T *recvbuf;
  size_t recvoffset;
  size_t count;
  int sendid;
  std::vector<int> recvids;
  BROADCAST(T *sb, size_t so, T *rb, size_t ro, size_t c, int sid, std::vector<int> ids)
      : sendbuf(sb), sendoffset(so), recvbuf(rb), recvoffset(ro), count(c), sendid(sid), recvids(std::move(ids)) {}
};

// One level of a schedule on one library: transfers + computes (coll.h).
template <typename T>
struct Coll {
  struct Xfer {
    T *sendbuf;
    size_t sendoffset;
    T *recvbuf;
    size_t recvoffset;
    size_t count;
    int sendid, recvid;
    bool feeds;  // the receive buffer exists only to feed a compute of the same level
  };
  struct Comp {
    std::vector<T *> inputs;
    T *output;
    size_t count;
    int compid;
  };
  CommBench::library lib;
  std::vector<Xfer> xfers;
  std::vector<Comp> comps;

  explicit Coll(CommBench::library l) : lib(l) {}
  void add(T *sb, size_t so, T *rb, size_t ro, size_t c, int sid, int rid, bool feeds = false) {
    xfers.push_back({sb, so, rb, ro, c, sid, rid, feeds});
  }
  void add(std::vector<T *> in, T *out, size_t c, int compid) { comps.push_back({std::move(in), out, c, compid}); }
  int numcomm() const { return (int)xfers.size(); }
  int numcompute() const { return (int)comps.size(); }
  bool empty() const { return xfers.empty() && comps.empty(); }

  // coll.h:46-94 style summary (printed by the print rank only; counts are
  // global because every rank holds every entry).
  void report(int np) const {
    std::printf("%s: %d transfers", CommBench::lib_name(lib), numcomm());
    size_t bytes = 0;
    for (auto &x : xfers) bytes += x.count * sizeof(T);
    std::printf(" (");
    CommBench::print_data(bytes);
    std::printf(")");
    if (!comps.empty()) {
      std::vector<int> fanin(np, 0), outs(np, 0);
      for (auto &c : comps) {
        fanin[c.compid] += (int)c.inputs.size();
        outs[c.compid]++;
      }
      std::printf(", %d computes:", numcompute());
      for (int p = 0; p < np && np < 64; p++)
        if (outs[p]) std::printf(" %d:%d->%d", p, fanin[p], outs[p]);
    }
    std::printf("\n");
  }
};

template <typename T>
using CollList = std::list<Coll<T> *>;

template <typename T>
class Planner {
 public:
  using Alloc = std::function<T *(size_t)>;
  int me, np;
  size_t buffsize = 0, recycle = 0, reuse = 0;  // elements (hiccl.h:36-38 counters)

  Planner(int me_, int np_, Alloc alloc) : me(me_), np(np_), alloc_(std::move(alloc)) {}

  // ------------------------------------------------------------- reduce --

  // Receive buffers of one tree invocation, reused level after level
  // (reduce.h:139-155), per rank.
  struct Pool {
    std::vector<std::pair<T *, size_t>> slots;
    size_t next = 0;
  };

  // reduce.h:69-211.  Levels from `level` down to 0; groups of gsz[level]
  // ranks each reduce to the member at the receiver's position.
  void reduce_tree(int numlevel, const int *gsz, const CommBench::library *lib, std::vector<REDUCE<T>> list,
                   int level, CollList<T> &out, Pool &pool) {
    if (list.empty() || level < 0) return;
    auto *coll = new Coll<T>(lib[level]);
    std::vector<REDUCE<T>> up;
    const int gs = gsz[level];
    pool.next = 0;
    for (auto &r : list) {
      std::vector<int> heads;
      T *mine = nullptr;
      size_t mine_off = 0;
      for (int g = 0; g < np / gs; g++) {
        std::vector<int> members;
        for (int s : r.sendids)
          if (s / gs == g) members.push_back(s);
        if (members.empty()) continue;
        const int head = g * gs + r.recvid % gs;
        T *obuf = nullptr;
        size_t ooff = 0;
        auto output = [&]() {  // the final receiver writes in place, others get a buffer
          if (head == r.recvid) {
            obuf = r.recvbuf;
            ooff = r.recvoffset;
            if (me == head) reuse += r.count;
          } else {
            obuf = take(head, r.count);
          }
        };
        if (members.size() > 1) {
          output();
          std::vector<T *> inputs;
          for (int s : members) {
            if (s == head) {
              inputs.push_back(at(r.sendbuf, r.sendoffset));
            } else {
              T *rb = pooled(head, r.count, pool);
              coll->add(r.sendbuf, r.sendoffset, rb, 0, r.count, s, head, true);
              inputs.push_back(rb);
            }
          }
          coll->add(std::move(inputs), at(obuf, ooff), r.count, head);
        } else if (members[0] != head || level == numlevel - 1) {
          output();
          coll->add(r.sendbuf, r.sendoffset, obuf, ooff, r.count, members[0], head);
        } else {  // the head alone holds the data: pass its buffer up
          obuf = r.sendbuf;
          ooff = r.sendoffset;
        }
        heads.push_back(head);
        if (me == head) {
          mine = obuf;
          mine_off = ooff;
        }
      }
      if (!heads.empty()) up.emplace_back(mine, mine_off, r.recvbuf, r.recvoffset, r.count, heads, r.recvid);
    }
    keep(coll, out);
    reduce_tree(numlevel, gsz, lib, std::move(up), level - 1, out, pool);
  }

  // reduce.h:213-335.  Reduces with senders on other nodes send the partial
  // of the next node along the ring; the recursion's colls precede this
  // step's, and the recursion ends in the intra-node tree.
  void reduce_ring(int numlevel, const int *gsz, const CommBench::library *lib, std::vector<REDUCE<T>> &list,
                   std::vector<REDUCE<T>> &intra, CollList<T> &out) {
    std::vector<REDUCE<T>> further;
    auto *coll = new Coll<T>(lib[0]);
    const int gs0 = gsz[0], numnode = np / gs0;
    for (auto &r : list) {
      const int rnode = r.recvid / gs0;
      std::vector<int> local, remote;
      for (int s : r.sendids) (s / gs0 == rnode ? local : remote).push_back(s);
      if (remote.empty()) {
        intra.push_back(r);
        continue;
      }
      const int snode = (rnode + 1) % numnode;
      const int fwd = snode * gs0 + r.recvid % gs0;  // forwards the ring partial
      std::vector<std::vector<int>> by_node(numnode);
      for (int s : r.sendids) by_node[s / gs0].push_back(s);
      size_t beyond = 0;
      for (int node = 0; node < numnode; node++)
        if (node != rnode && node != snode) beyond += by_node[node].size();
      T *part;
      size_t part_off = 0;
      if (by_node[snode].size() == 1 && by_node[snode][0] == fwd && beyond == 0) {
        part = r.sendbuf;  // the forwarding rank's own data is the whole partial
        part_off = r.sendoffset;
        by_node[snode].clear();
        if (me == fwd) reuse += r.count;
      } else {
        part = take(fwd, r.count);
      }
      std::vector<int> rest;
      for (int node = 0; node < numnode; node++)
        if (node != rnode) rest.insert(rest.end(), by_node[node].begin(), by_node[node].end());
      further.emplace_back(r.sendbuf, r.sendoffset, part, part_off, r.count, rest, fwd);
      T *land;
      size_t land_off = 0;
      if (local.empty()) {
        land = r.recvbuf;
        land_off = r.recvoffset;
        if (me == r.recvid) reuse += r.count;
      } else {
        land = take(r.recvid, r.count);
        T *mine = take(r.recvid, r.count);
        intra.emplace_back(r.sendbuf, r.sendoffset, mine, 0, r.count, local, r.recvid);
        coll->add(std::vector<T *>{land, mine}, at(r.recvbuf, r.recvoffset), r.count, r.recvid);
      }
      // when `part` is the forwarding rank's own send buffer, `further`
      // holds an empty reduce and this transfer moves the raw data
      T *src = part;
      size_t src_off = part_off;
      if (me != fwd) src = nullptr;
      coll->add(src, src_off, land, land_off, r.count, fwd, r.recvid, !local.empty());
    }
    if (!further.empty()) {
      reduce_ring(numlevel, gsz, lib, further, intra, out);
    } else {
      std::vector<int> gt(gsz, gsz + numlevel);
      gt[0] = np;
      Pool pool;
      reduce_tree(numlevel, gt.data(), lib, intra, numlevel - 1, out, pool);
    }
    keep(coll, out);
  }

  // reduce.h:337-399: reduces with senders outside the receiver's stripe
  // group are split over `numstripe` receivers; returns the multicasts that
  // deliver each stripe's result to the final receiver.
  std::vector<BROADCAST<T>> stripe(int numstripe, std::vector<REDUCE<T>> &list) {
    std::vector<BROADCAST<T>> merge;
    std::vector<REDUCE<T>> inter, result;
    for (auto &r : list) {
      bool cross = false;
      for (int s : r.sendids) cross = cross || (s / numstripe != r.recvid / numstripe);
      (cross ? inter : result).push_back(r);
    }
    for (auto &r : inter) {
      const int node = r.recvid / numstripe;
      size_t off = 0;
      for (int st = 0; st < numstripe; st++) {
        const size_t cnt = r.count / numstripe + ((size_t)st < r.count % numstripe ? 1 : 0);
        if (!cnt) break;
        const int recver = node * numstripe + st;
        T *rb;
        size_t ro = 0;
        if (recver != r.recvid) {
          rb = take(recver, cnt);
          merge.emplace_back(rb, 0, r.recvbuf, r.recvoffset + off, cnt, recver, std::vector<int>{r.recvid});
        } else {
          rb = r.recvbuf;
          ro = r.recvoffset + off;
          if (me == recver) reuse += cnt;
        }
        result.emplace_back(r.sendbuf, r.sendoffset + off, rb, ro, cnt, r.sendids, recver);
        off += cnt;
      }
    }
    list.swap(result);
    return merge;
  }

  // ---------------------------------------------------------- broadcast --

  // broadcast.h:69-172: outermost level first; the leaf level delivers.
  void bcast_tree(int numlevel, const int *gsz, const CommBench::library *lib, std::vector<BROADCAST<T>> list,
                  int level, CollList<T> &out) {
    if (list.empty()) return;
    auto *coll = new Coll<T>(lib[level - 1]);
    std::vector<BROADCAST<T>> down;
    if (level == numlevel) {
      for (auto &b : list)
        for (int r : b.recvids) coll->add(b.sendbuf, b.sendoffset, b.recvbuf, b.recvoffset, b.count, b.sendid, r);
    } else {
      const int gs = gsz[level];
      for (auto &b : list) {  // receivers in the sender's own group
        std::vector<int> ids;
        for (int r : b.recvids)
          if (r / gs == b.sendid / gs) ids.push_back(r);
        if (!ids.empty()) down.emplace_back(b.sendbuf, b.sendoffset, b.recvbuf, b.recvoffset, b.count, b.sendid, ids);
      }
      for (int g = 0; g < np / gs; g++) {  // one representative per other group
        for (auto &b : list) {
          if (b.sendid / gs == g) continue;
          std::vector<int> ids;
          for (int r : b.recvids)
            if (r / gs == g) ids.push_back(r);
          if (ids.empty()) continue;
          const int rep = g * gs + b.sendid % gs;
          T *land;
          size_t loff = 0;
          auto it = std::find(ids.begin(), ids.end(), rep);
          if (it != ids.end()) {
            ids.erase(it);
            land = b.recvbuf;
            loff = b.recvoffset;
            if (me == rep) reuse += b.count;
          } else {
            land = take(rep, b.count);
          }
          coll->add(b.sendbuf, b.sendoffset, land, loff, b.count, b.sendid, rep);
          if (!ids.empty()) down.emplace_back(land, loff, b.recvbuf, b.recvoffset, b.count, rep, ids);
        }
      }
    }
    keep(coll, out);
    bcast_tree(numlevel, gsz, lib, std::move(down), level + 1, out);
  }

  // broadcast.h:174-236: hop to the same position on the next node; this
  // step's coll precedes the recursion's.
  void bcast_ring(int gs0, CommBench::library lib0, std::vector<BROADCAST<T>> &list, std::vector<BROADCAST<T>> &intra,
                  CollList<T> &out) {
    std::vector<BROADCAST<T>> further;
    auto *coll = new Coll<T>(lib0);
    const int numnode = np / gs0;
    for (auto &b : list) {
      const int snode = b.sendid / gs0;
      std::vector<int> local, remote;
      for (int r : b.recvids) (r / gs0 == snode ? local : remote).push_back(r);
      if (!local.empty()) intra.emplace_back(b.sendbuf, b.sendoffset, b.recvbuf, b.recvoffset, b.count, b.sendid, local);
      if (remote.empty()) continue;
      const int rep = ((snode + 1) % numnode) * gs0 + b.sendid % gs0;
      T *land;
      size_t loff = 0;
      auto it = std::find(remote.begin(), remote.end(), rep);
      if (it != remote.end()) {
        remote.erase(it);
        land = b.recvbuf;
        loff = b.recvoffset;
        if (me == rep) reuse += b.count;
      } else {
        land = take(rep, b.count);
      }
      coll->add(b.sendbuf, b.sendoffset, land, loff, b.count, b.sendid, rep);
      if (!remote.empty()) further.emplace_back(land, loff, b.recvbuf, b.recvoffset, b.count, rep, remote);
    }
    keep(coll, out);
    if (!further.empty()) bcast_ring(gs0, lib0, further, intra, out);
  }

  // broadcast.h:238-319: multicasts leaving the sender's stripe group are
  // split over numstripe senders, each first fed by a direct transfer
  // (returned as single-sender reduces).
  std::vector<REDUCE<T>> stripe(int numstripe, std::vector<BROADCAST<T>> &list) {
    std::vector<REDUCE<T>> split;
    std::vector<BROADCAST<T>> inter, result;
    for (auto &b : list) {
      bool cross = false;
      for (int r : b.recvids) cross = cross || (r / numstripe != b.sendid / numstripe);
      (cross ? inter : result).push_back(b);
    }
    for (auto &b : inter) {
      const int group = b.sendid / numstripe;
      size_t off = 0;
      for (int st = 0; st < numstripe; st++) {
        const size_t cnt = b.count / numstripe + ((size_t)st < b.count % numstripe ? 1 : 0);
        if (!cnt) break;
        const int sender = group * numstripe + st;
        std::vector<int> ids = b.recvids;
        T *sb;
        size_t so = 0;
        if (sender != b.sendid) {
          auto it = std::find(ids.begin(), ids.end(), sender);
          if (it != ids.end()) {
            ids.erase(it);
            sb = b.recvbuf;
            so = b.recvoffset + off;
            if (me == sender) reuse += cnt;
          } else {
            sb = take(sender, cnt);
          }
          split.emplace_back(b.sendbuf, b.sendoffset + off, sb, so, cnt, std::vector<int>{b.sendid}, sender);
        } else {
          sb = b.sendbuf;
          so = b.sendoffset + off;
          if (me == sender) reuse += cnt;
        }
        result.emplace_back(sb, so, b.recvbuf, b.recvoffset + off, cnt, sender, ids);
        off += cnt;
      }
    }
    list.swap(result);
    return split;
  }

 private:
  Alloc alloc_;

  T *take(int owner, size_t n) {
    if (owner != me) return nullptr;
    buffsize += n;
    return alloc_(n);
  }

  T *pooled(int owner, size_t n, Pool &pool) {
    if (owner != me) return nullptr;
    if (pool.next < pool.slots.size() && pool.slots[pool.next].second >= n) {
      recycle += n;
      return pool.slots[pool.next++].first;
    }
    T *p = take(owner, n);
    if (pool.next < pool.slots.size())
      pool.slots[pool.next] = {p, n};
    else
      pool.slots.push_back({p, n});
    pool.next++;
    return p;
  }

  static void keep(Coll<T> *c, CollList<T> &out) {
    if (c->empty())
      delete c;
    else
      out.push_back(c);
  }
};

// reduce.h:401-415 / broadcast.h:321-335: split every primitive into
// `numbatch` consecutive pieces (count/numbatch, the first count%numbatch
// pieces one element longer), stopping at the first empty piece.
template <typename P>
std::vector<std::vector<P>> partition(const std::vector<P> &list, int numbatch) {
  std::vector<std::vector<P>> out(numbatch);
  for (auto &p : list) {
    size_t off = 0;
    for (int b = 0; b < numbatch; b++) {
      const size_t cnt = p.count / numbatch + ((size_t)b < p.count % numbatch ? 1 : 0);
      if (!cnt) break;
      P q = p;
      q.sendoffset += off;
      q.recvoffset += off;
      q.count = cnt;
      out[b].push_back(q);
      off += cnt;
    }
  }
  return out;
}

}  // namespace HiCCL

#endif  // HICCL_PLAN_H
