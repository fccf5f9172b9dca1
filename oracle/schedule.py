"""oracle/schedule.py -- TEST INFRASTRUCTURE ONLY.

Python restatement of HiCCL's schedule factorization (reference @ 2024-12-20)
and a numpy simulator that executes the resulting plan for every rank.  It is
the checker for SURVEY.md section 8 rows a7-a12 (which computes exist, their
input ORDER, counts and offsets, and the step structure), never product code.

Restated (file:line in /root/reference/source):
  REDUCE / BROADCAST pattern expansion   reduce.h:51-66, broadcast.h:52-66
  reduce_tree                            reduce.h:69-211
  reduce_ring                            reduce.h:213-335
  stripe (reduce / bcast)                reduce.h:337-399, broadcast.h:238-319
  partition (reduce / bcast)             reduce.h:401-415, broadcast.h:321-335
  bcast_tree / bcast_ring                broadcast.h:69-172, broadcast.h:174-236
  init (per epoch: bcast then reduce)    init.h:2-76
  groupsize from the hierarchy           comm.h:160-179 (init())
  implement (stagger + merge per lib)    command.h:40-165
  run (comm start; reverse-lib wait +
       compute start; compute wait)      comm.h:181-206

The reference's SPMD pointers (valid only on the owning rank) are modelled
symbolically: a location is (rank, buffer_key, element_offset); user buffers
are ("send",) / ("recv",) per rank; temporaries are ("tmp", owner, serial).
Receive-buffer recycling (reduce.h:139-155) only saves memory and is not
modelled (every temporary is fresh), which cannot change any value.
"""
import numpy as np

# CommBench::library order (hiccl.h uses these names)
DUMMY, IPC, IPC_GET, MPI, XCCL, NUMLIB = range(6)


class Reduce:
    """REDUCE<T> (reduce.h:2-67).  send: {rank: (buf, off)}; recv on recvid."""

    def __init__(self, send, recv, count, sendids, recvid):
        self.send = dict(send)
        self.recv = recv
        self.count = count
        self.sendids = list(sendids)
        self.recvid = recvid


class Bcast:
    """BROADCAST<T> (broadcast.h:2-67).  send on sendid; recv: (buf, off) on every receiver."""

    def __init__(self, send, recv, count, sendid, recvids):
        self.send = send
        self.recv = recv
        self.count = count
        self.sendid = sendid
        self.recvids = list(recvids)


def expand_ids(pattern_id, numproc, other):
    """reduce.h:54-66 / broadcast.h:54-66: numproc -> all ranks ascending,
    -1 -> all but `other`, else the single id."""
    if pattern_id == numproc:
        return list(range(numproc))
    if pattern_id == -1:
        return [i for i in range(numproc) if i != other]
    return [i for i in range(numproc) if i == pattern_id]


class Coll:
    """Coll<T> (coll.h:1-95): one level's transfers + computes on one library."""

    def __init__(self, lib):
        self.lib = lib
        self.comms = []      # (src_rank, (buf, off), dst_rank, (buf, off), count)
        self.computes = []   # (rank, [(buf, off), ...], (buf, off), count)

    def add_comm(self, src_rank, src, dst_rank, dst, count):
        self.comms.append((src_rank, src, dst_rank, dst, count))

    def add_compute(self, rank, inputs, out, count):
        self.computes.append((rank, list(inputs), out, count))

    def empty(self):
        return not self.comms and not self.computes


class Planner:
    def __init__(self, numproc, ring_reuse_fix=False):
        self.numproc = numproc
        self._tmp = 0
        # The reference reuses the next ring node's send buffer as the ring
        # partial whenever that node's only sender is the forwarding rank
        # (reduce.h:261-270), even if further nodes are then reduced INTO it
        # (overwriting user data, dropping that rank's term).  False restates
        # the reference as is; True reuses it only when no node lies beyond,
        # which is what the build does (include/hiccl/plan.h).
        self.ring_reuse_fix = ring_reuse_fix

    def alloc(self, rank):
        self._tmp += 1
        return ("tmp", rank, self._tmp)

    # ------------------------------------------------------------ reduce --
    def reduce_tree(self, numlevel, groupsize, lib, reducelist, level, coll_list):
        """reduce.h:69-211 (innermost level first, recursing level-1)."""
        if not reducelist or level == -1:
            return
        coll = Coll(lib[level])
        new = []
        numgroup = self.numproc // groupsize[level]
        for red in reducelist:
            ids_new, send_new = [], {}
            for g in range(numgroup):
                ids = [s for s in red.sendids if s // groupsize[level] == g]
                if not ids:
                    continue
                recvid = g * groupsize[level] + red.recvid % groupsize[level]
                if recvid == red.recvid:
                    out = red.recv
                else:
                    out = (self.alloc(recvid), 0)
                if len(ids) > 1:
                    inputs = []
                    for s in ids:
                        if s != recvid:
                            rb = (self.alloc(recvid), 0)
                            coll.add_comm(s, red.send[s], recvid, rb, red.count)
                            inputs.append(rb)
                        else:
                            inputs.append(red.send[s])
                    coll.add_compute(recvid, inputs, out, red.count)
                else:
                    s = ids[0]
                    if s != recvid:
                        coll.add_comm(s, red.send[s], recvid, out, red.count)
                    elif level == numlevel - 1:
                        coll.add_comm(s, red.send[s], recvid, out, red.count)
                    else:
                        out = red.send[s]
                ids_new.append(recvid)
                send_new[recvid] = out
            if ids_new:
                new.append(Reduce(send_new, red.recv, red.count, ids_new, red.recvid))
        if not coll.empty():
            coll_list.append(coll)
        self.reduce_tree(numlevel, groupsize, lib, new, level - 1, coll_list)

    def reduce_ring(self, numlevel, groupsize, lib, reducelist, intra, coll_list):
        """reduce.h:213-335.  The recursion's colls come BEFORE this step's."""
        extra_list = []
        coll = Coll(lib[0])
        gs0 = groupsize[0]
        for red in reducelist:
            recvnode = red.recvid // gs0
            ids_intra = [s for s in red.sendids if s // gs0 == recvnode]
            ids_extra = [s for s in red.sendids if s // gs0 != recvnode]
            if not ids_extra:
                intra.append(Reduce(red.send, red.recv, red.count, red.sendids, red.recvid))
                continue
            numnode = self.numproc // gs0
            sendnode = (numnode + recvnode + 1) % numnode
            by_node = [[] for _ in range(numnode)]
            for s in red.sendids:
                by_node[s // gs0].append(s)
            sendid = sendnode * gs0 + red.recvid % gs0
            beyond = sum(len(by_node[nd]) for nd in range(numnode) if nd not in (recvnode, sendnode))
            if by_node[sendnode] == [sendid] and not (self.ring_reuse_fix and beyond):
                ring_src = red.send[sendid]
                by_node[sendnode] = []
            else:
                ring_src = (self.alloc(sendid), 0)
            rest = [s for node in range(numnode) if node != recvnode for s in by_node[node]]
            extra_list.append(Reduce(red.send, ring_src, red.count, rest, sendid))
            if not ids_intra:
                land = red.recv
            else:
                land = (self.alloc(red.recvid), 0)
                part = (self.alloc(red.recvid), 0)
                intra.append(Reduce(red.send, part, red.count, ids_intra, red.recvid))
                coll.add_compute(red.recvid, [land, part], red.recv, red.count)
            coll.add_comm(sendid, ring_src, red.recvid, land, red.count)
        if extra_list:
            self.reduce_ring(numlevel, groupsize, lib, extra_list, intra, coll_list)
        else:
            gt = list(groupsize)
            gt[0] = self.numproc
            self.reduce_tree(numlevel, gt, lib, intra, numlevel - 1, coll_list)
        if not coll.empty():
            coll_list.append(coll)

    def stripe_reduce(self, numstripe, reducelist):
        """reduce.h:337-399 (in place); returns the merge list (Bcasts)."""
        nodesize = numstripe
        intra_l, inter_l = [], []
        for red in reducelist:
            inter = [s for s in red.sendids if s // nodesize != red.recvid // nodesize]
            (inter_l if inter else intra_l).append(red)
        merge = []
        reducelist[:] = list(intra_l)
        for red in inter_l:
            recvnode = red.recvid // nodesize
            off = 0
            for st in range(numstripe):
                recver = recvnode * nodesize + st
                cnt = red.count // numstripe + (1 if st < red.count % numstripe else 0)
                if not cnt:
                    break
                if recver != red.recvid:
                    land = (self.alloc(recver), 0)
                    merge.append(Bcast(land, (red.recv[0], red.recv[1] + off), cnt, recver, [red.recvid]))
                else:
                    land = (red.recv[0], red.recv[1] + off)
                send = {r: (b, o + off) for r, (b, o) in red.send.items()}
                reducelist.append(Reduce(send, land, cnt, red.sendids, recver))
                off += cnt
        return merge

    # ------------------------------------------------------------- bcast --
    def bcast_tree(self, numlevel, groupsize, lib, bcastlist, level, coll_list):
        """broadcast.h:69-172 (outermost level first, recursing level+1)."""
        if not bcastlist:
            return
        coll = Coll(lib[level - 1])
        new = []
        if level == numlevel:
            for b in bcastlist:
                for r in b.recvids:
                    coll.add_comm(b.sendid, b.send, r, b.recv, b.count)
        else:
            gsl = groupsize[level]
            numgroup = self.numproc // gsl
            for b in bcastlist:
                sg = b.sendid // gsl
                ids = [r for r in b.recvids if r // gsl == sg]
                if ids:
                    new.append(Bcast(b.send, b.recv, b.count, b.sendid, ids))
            for rg in range(numgroup):
                for b in bcastlist:
                    if b.sendid // gsl == rg:
                        continue
                    ids = [r for r in b.recvids if r // gsl == rg]
                    if not ids:
                        continue
                    rep = rg * gsl + b.sendid % gsl
                    if rep in ids:
                        land = b.recv
                        ids.remove(rep)
                    else:
                        land = (self.alloc(rep), 0)
                    coll.add_comm(b.sendid, b.send, rep, land, b.count)
                    if ids:
                        new.append(Bcast(land, b.recv, b.count, rep, ids))
        if not coll.empty():
            coll_list.append(coll)
        self.bcast_tree(numlevel, groupsize, lib, new, level + 1, coll_list)

    def bcast_ring(self, gs0, lib0, bcastlist, intra, coll_list):
        """broadcast.h:174-236 (this step's coll BEFORE the recursion's)."""
        extra_l = []
        coll = Coll(lib0)
        numnode = self.numproc // gs0
        for b in bcastlist:
            sendnode = b.sendid // gs0
            ids_in = [r for r in b.recvids if r // gs0 == sendnode]
            ids_ex = [r for r in b.recvids if r // gs0 != sendnode]
            if ids_in:
                intra.append(Bcast(b.send, b.recv, b.count, b.sendid, ids_in))
            if ids_ex:
                rep = ((sendnode + 1) % numnode) * gs0 + b.sendid % gs0
                if rep in ids_ex:
                    ids_ex.remove(rep)
                    land = b.recv
                else:
                    land = (self.alloc(rep), 0)
                coll.add_comm(b.sendid, b.send, rep, land, b.count)
                if ids_ex:
                    extra_l.append(Bcast(land, b.recv, b.count, rep, ids_ex))
        if not coll.empty():
            coll_list.append(coll)
        if extra_l:
            self.bcast_ring(gs0, lib0, extra_l, intra, coll_list)

    def stripe_bcast(self, numstripe, bcastlist):
        """broadcast.h:238-319 (in place); returns the split list (Reduces)."""
        nodesize = numstripe
        intra_l, inter_l = [], []
        for b in bcastlist:
            inter = [r for r in b.recvids if r // nodesize != b.sendid // nodesize]
            (inter_l if inter else intra_l).append(b)
        split = []
        bcastlist[:] = list(intra_l)
        for b in inter_l:
            sg = b.sendid // nodesize
            off = 0
            for st in range(numstripe):
                sender = sg * nodesize + st
                cnt = b.count // numstripe + (1 if st < b.count % numstripe else 0)
                if not cnt:
                    break
                ids = list(b.recvids)
                if sender != b.sendid:
                    if sender in ids:
                        ids.remove(sender)
                        src = (b.recv[0], b.recv[1] + off)
                    else:
                        src = (self.alloc(sender), 0)
                    split.append(Reduce({b.sendid: (b.send[0], b.send[1] + off)}, src, cnt, [b.sendid], sender))
                else:
                    src = (b.send[0], b.send[1] + off)
                bcastlist.append(Bcast(src, (b.recv[0], b.recv[1] + off), cnt, sender, ids))
                off += cnt
        return split


def partition(prims, numbatch):
    """reduce.h:401-415 / broadcast.h:321-335."""
    batches = [[] for _ in range(numbatch)]
    for p in prims:
        off = 0
        for b in range(numbatch):
            cnt = p.count // numbatch + (1 if b < p.count % numbatch else 0)
            if not cnt:
                break
            if isinstance(p, Reduce):
                send = {r: (bf, o + off) for r, (bf, o) in p.send.items()}
                batches[b].append(Reduce(send, (p.recv[0], p.recv[1] + off), cnt, p.sendids, p.recvid))
            else:
                batches[b].append(Bcast((p.send[0], p.send[1] + off), (p.recv[0], p.recv[1] + off), cnt,
                                        p.sendid, p.recvids))
            off += cnt
    return batches


def groupsizes(hierarchy, numproc, ringnodes):
    """comm.h:160-179."""
    L = len(hierarchy)
    gs = [0] * L
    gs[L - 1] = hierarchy[L - 1]
    for i in range(L - 2, -1, -1):
        gs[i] = gs[i + 1] * hierarchy[i]
    gs[0] = numproc // ringnodes
    return gs


class Schedule:
    """Comm<T> (comm.h) restated: epochs of primitives -> steps."""

    def __init__(self, numproc, hierarchy=None, libs=None, numstripe=1, ringnodes=1, pipedepth=1,
                 ring_reuse_fix=False):
        self.numproc = numproc
        self.ring_reuse_fix = ring_reuse_fix
        self.hierarchy = hierarchy or [numproc]
        self.libs = libs or [MPI] * len(self.hierarchy)
        self.numstripe = numstripe
        self.ringnodes = ringnodes
        self.pipedepth = pipedepth
        self.epochs = [([], [])]  # (bcasts, reduces); the ctor opens epoch 0 (comm.h:120-128)

    def add_fence(self):
        self.epochs.append(([], []))

    def add_reduce(self, sendbuf, sendoffset, recvbuf, recvoffset, count, sendids, recvid):
        """sendids: list, or an int pattern id (numproc = all, -1 = others)."""
        if isinstance(sendids, int):
            sendids = expand_ids(sendids, self.numproc, recvid)
        send = {r: ((sendbuf,), sendoffset) for r in range(self.numproc)}
        self.epochs[-1][1].append(Reduce(send, ((recvbuf,), recvoffset), count, sendids, recvid))

    def add_bcast(self, sendbuf, sendoffset, recvbuf, recvoffset, count, sendid, recvids):
        if isinstance(recvids, int):
            recvids = expand_ids(recvids, self.numproc, sendid)
        self.epochs[-1][0].append(Bcast(((sendbuf,), sendoffset), ((recvbuf,), recvoffset), count, sendid,
                                        recvids))

    def init(self):
        """init.h:2-76 + command.h implement(coll_batch, pipeline, 1)."""
        P = Planner(self.numproc, self.ring_reuse_fix)
        L = len(self.hierarchy)
        gs = groupsizes(self.hierarchy, self.numproc, self.ringnodes)
        gt = list(gs)
        gt[0] = self.numproc
        nb = self.pipedepth
        coll_batch = [[] for _ in range(nb)]
        for bcasts, reduces in self.epochs:
            if bcasts:
                bb = partition(bcasts, nb)
                for b in range(nb):
                    split = P.stripe_bcast(self.numstripe, bb[b])
                    P.reduce_tree(1, gt, [self.libs[L - 1]], split, 0, coll_batch[b])
                    intra = []
                    P.bcast_ring(gs[0], self.libs[0], bb[b], intra, coll_batch[b])
                    P.bcast_tree(L, gt, self.libs, intra, 1, coll_batch[b])
            if reduces:
                rb = partition(reduces, nb)
                for b in range(nb):
                    merge = P.stripe_reduce(self.numstripe, rb[b])
                    intra = []
                    P.reduce_ring(L, gs, self.libs, rb[b], intra, coll_batch[b])
                    P.bcast_tree(L, gt, self.libs, merge, 1, coll_batch[b])
        self.steps = implement(coll_batch, pipeoffset=1)
        return self.steps


def implement(coll_batch, pipeoffset=1):
    """command.h:40-165: batch i is delayed by i*pipeoffset dummy steps; the
    colls of all batches at one step are merged per library; steps with no
    work are dropped.  Returns [ {lib: Coll} ] in execution order."""
    used = sorted({c.lib for batch in coll_batch for c in batch})
    staggered = [[None] * (i * pipeoffset) + list(batch) for i, batch in enumerate(coll_batch)]
    steps = []
    depth = max((len(b) for b in staggered), default=0)
    for s in range(depth):
        merged = {lib: Coll(lib) for lib in used}
        any_work = False
        for b in staggered:
            if s < len(b) and b[s] is not None:
                c = b[s]
                merged[c.lib].comms.extend(c.comms)
                merged[c.lib].computes.extend(c.computes)
                any_work = any_work or not c.empty()
        if any_work:
            steps.append(merged)
    return steps


class Remote(tuple):
    """A compute input read in place on another rank (fused gather +
    reduce: the transfer that fed this input was dropped).  Remote((rank, loc))."""


def simulate(steps, numproc, user, dtype=np.float32):
    """Execute the plan.  user: {(rank, name): array}.  Temporaries are
    created on first write.  Comms of a step run before its computes (the
    reference's run(): every library's comm waits before that library's
    compute starts, and distinct batches of a step never touch the same
    bytes).  A compute is reduce_kernel: acc = 0; acc += in[k] in list order."""
    mem = {k: v.copy() for k, v in user.items()}

    def view(rank, loc, count):
        buf, off = loc
        key = (rank, buf)
        if key not in mem:  # temporaries start as NaN: reading one before it is written shows
            mem[key] = np.full(max(off + count, 1), np.nan, dtype)
        arr = mem[key]
        if len(arr) < off + count:
            arr = np.concatenate([arr, np.full(off + count - len(arr), np.nan, dtype)])
            mem[key] = arr
        return arr, off

    with np.errstate(all="ignore"):
        for step in steps:
            for lib in sorted(step):
                for (sr, src, dr, dst, cnt) in step[lib].comms:
                    sa, so = view(sr, src, cnt)
                    da, do = view(dr, dst, cnt)
                    da[do:do + cnt] = sa[so:so + cnt]
            for lib in sorted(step, reverse=True):
                for (r, ins, out, cnt) in step[lib].computes:
                    acc = np.zeros(cnt, dtype)
                    for loc in ins:
                        a, o = view(*loc, cnt) if isinstance(loc, Remote) else view(r, loc, cnt)
                        acc = (acc + a[o:o + cnt]).astype(dtype)
                    oa, oo = view(r, out, cnt)
                    oa[oo:oo + cnt] = acc
    return mem


def compose(pattern, numproc, count, root=0):
    """The collective compositions of collectives/main.cpp:104-160 on
    buffers ('send', 'recv'); returns a configured Schedule-builder fn."""
    def build(sch):
        if pattern == "gather":
            for s in range(numproc):
                sch.add_bcast("send", 0, "recv", s * count, count, s, root)
        elif pattern == "scatter":
            for r in range(numproc):
                sch.add_reduce("send", r * count, "recv", 0, count, root, r)
        elif pattern == "broadcast":
            sch.add_bcast("send", 0, "recv", 0, count * numproc, root, numproc)
        elif pattern == "reduce":
            sch.add_reduce("send", 0, "recv", 0, count * numproc, numproc, root)
        elif pattern == "alltoall":
            for s in range(numproc):
                for r in range(numproc):
                    sch.add_bcast("send", r * count, "recv", s * count, count, s, r)
        elif pattern == "allgather":
            for s in range(numproc):
                sch.add_bcast("send", 0, "recv", s * count, count, s, numproc)
        elif pattern == "reducescatter":
            for r in range(numproc):
                sch.add_reduce("send", r * count, "recv", 0, count, numproc, r)
        elif pattern == "allreduce":
            for r in range(numproc):
                sch.add_reduce("send", r * count, "recv", r * count, count, numproc, r)
            sch.add_fence()
            for s in range(numproc):
                sch.add_bcast("recv", s * count, "recv", s * count, count, s, -1)
        else:
            raise ValueError(pattern)
    return build


PATTERN_IDS = {"gather": 1, "scatter": 2, "broadcast": 3, "reduce": 4, "alltoall": 5, "allgather": 6,
               "reducescatter": 7, "allreduce": 8}  # hiccl.h:41 enum collective
