"""Branch-level concurrency of the Inception step: lanes (HIP streams) and
the event dependencies between them.

An Inception block runs 3-4 independent branches between its input buffer
and its concat-free output slices, and from mixed4 on the
branch layers are small (17x17, 8x8 at batch 64): a few hundred workgroups
and a few microseconds each, latency- rather than throughput-bound on 256
CUs.  Running the branches on separate streams lets the hardware overlap
them (inside a captured HIP graph the cross-stream event waits become graph
edges).

* node_lanes: a launch that reads a buffer written by exactly one launch
  continues that launch's lane (the first such reader does; further readers
  of the same producer fork onto new lanes); readers of block buffers (several
  producers: the concat-free block outputs) start new lanes round-robin.
  Backward calls of a node run on its forward lane.
* schedule: every call declares the resources it reads and writes
  (activation / gradient channel slices, raw outputs and statistics of a
  launch, per-launch gradient regions, per-lane scratch, ...).  Over the
  whole step's call sequence (forward, backward, update in issue order) each
  call waits for the last writer of what it reads or writes and for the
  readers since that write of what it writes (RAW, WAW, WAR) -- when those run
  on another lane (by waiting for that lane's tail); same-lane order is
  stream order.  (Eager runs wait for the producing call itself instead of
  the other lane's tail: Call.pwaits.)  Accumulating writers of
  one gradient buffer are therefore serialised in issue order, so the result
  is bitwise the single-stream result.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple


@dataclass
class Call:
    fn: object
    args: tuple
    name: str
    lane: int = 0
    reads: Tuple = ()
    writes: Tuple = ()
    idx: int = -1                                   # position in the step's call sequence
    waits: List[int] = field(default_factory=list)  # lanes whose work so far must finish first
    nbytes: int = 0                                 # algorithmic HBM bytes (memory-bound ops; bench.py)
    # producer waits (eager runs): (lane, call index) pairs -- wait for THAT
    # call of the other lane (an event recorded right after it), not for
    # everything the host had issued there by then; record: this call is
    # such a producer
    pwaits: List[Tuple[int, int]] = field(default_factory=list)
    record: bool = False


def node_lanes(g, plan, nl: int) -> Dict[int, int]:
    """Graph node index -> lane in [0, nl)."""
    if nl <= 1:
        return {i: 0 for i in range(len(g.nodes))}
    index = {id(n): i for i, n in enumerate(g.nodes)}

    def launch_of(i):                      # node that issues node i's launch
        n = g.nodes[i]
        return index[id(plan.unit_of[n.idx].first)] if n.kind == "conv" else i

    producers: Dict[int, set] = {}
    for i, n in enumerate(g.nodes):
        producers.setdefault(n.y.buf, set()).add(launch_of(i))
    lane: Dict[int, int] = {}
    taken = set()
    rr = 0
    for i, n in enumerate(g.nodes):
        li = launch_of(i)
        if li != i:
            lane[i] = lane[li]
            continue
        p = producers.get(n.x, set())
        src = next(iter(p)) if len(p) == 1 else None
        if src is not None and src not in taken:
            taken.add(src)
            lane[i] = lane[src]
        else:
            lane[i] = rr % nl
            rr += 1
    return lane


def schedule(calls: Sequence[Call]) -> None:
    """Number the calls and fill in the lanes each must wait for.  A wait is
    on the TAIL of the other lane at issue time (an event recorded there just
    before the wait), which covers every call issued on that lane so far; a
    lane already waited for at a tail at or past the needed call is skipped.
    (Waiting on an event recorded earlier, while its stream has since moved
    on, made hipGraphInstantiate crash with three or more lanes on ROCm 7.2;
    tail events are also what the fork / join of a step use.)"""
    last_w: Dict[object, int] = {}
    readers: Dict[object, List[int]] = {}
    tail: Dict[int, int] = {}                       # lane -> newest call issued on it
    synced: Dict[Tuple[int, int], int] = {}         # (lane, other lane) -> other lane's tail when last waited for
    psynced: Dict[Tuple[int, int], int] = {}        # the same for the producer waits
    for i, c in enumerate(calls):
        c.idx = i
        c.waits = []
        c.pwaits = []
        c.record = False
    for i, c in enumerate(calls):
        dep = set()
        for k in c.reads:
            if k in last_w:
                dep.add(last_w[k])
        for k in c.writes:
            if k in last_w:
                dep.add(last_w[k])
            dep.update(readers.get(k, ()))
        for k in c.reads:
            readers.setdefault(k, []).append(i)
        for k in c.writes:
            last_w[k] = i
            readers[k] = []
        need: Dict[int, int] = {}
        for j in dep:
            lj = calls[j].lane
            if lj != c.lane:
                need[lj] = max(need.get(lj, -1), j)
        for lj, j in sorted(need.items()):
            if psynced.get((c.lane, lj), -1) < j:   # (a wait for j' >= j on lane lj covers j)
                psynced[(c.lane, lj)] = j
                c.pwaits.append((lj, j))
                calls[j].record = True
            if synced.get((c.lane, lj), -1) >= j:
                continue                            # already waited for a tail at or past j
            synced[(c.lane, lj)] = tail[lj]
            c.waits.append(lj)
        tail[c.lane] = i


def check_schedule(calls: Sequence[Call], precise: bool = False) -> None:
    """Test helper: every pair of conflicting calls on different lanes is
    ordered by a chain of same-lane order and tail waits (precise: producer
    waits) -- happens-before."""
    hb: List[Dict[int, int]] = []
    last_on_lane: Dict[int, int] = {}
    for i, c in enumerate(calls):
        known: Dict[int, int] = {}
        prev = last_on_lane.get(c.lane)
        if prev is not None:
            known = dict(hb[prev])
            known[c.lane] = max(known.get(c.lane, -1), prev)
        targets = ([(lj, j) for lj, j in c.pwaits] if precise
                   else [(lj, last_on_lane.get(lj)) for lj in c.waits])
        for lj, t in targets:
            assert lj != c.lane
            if t is None:
                continue
            if precise:
                assert calls[t].lane == lj and calls[t].record and t < i
            for l2, k in hb[t].items():
                known[l2] = max(known.get(l2, -1), k)
            known[lj] = max(known.get(lj, -1), t)
        hb.append(known)
        last_on_lane[c.lane] = i
    for i, ci in enumerate(calls):
        wi, ri = set(ci.writes), set(ci.reads)
        for j in range(i):
            cj = calls[j]
            if cj.lane == ci.lane:
                continue
            if (wi & (set(cj.writes) | set(cj.reads))) or (ri & set(cj.writes)):
                assert hb[i].get(cj.lane, -1) >= j, (cj.name, j, ci.name, i)
