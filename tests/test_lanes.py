"""jr.lanes on CPU: lane assignment follows the Inception branches, and the
event schedule orders every pair of conflicting calls on different lanes
(happens-before), on synthetic call sequences and on the structure of the
real step (resources as the engine declares them)."""
import random

from jr.inception import build_inception_v3
from jr.lanes import Call, check_schedule, node_lanes, schedule
from jr.plan import build_plan


def test_lanes_follow_branches():
    g = build_inception_v3()
    plan = build_plan(g)
    lane = node_lanes(g, plan, 4)
    assert set(lane.values()) == {0, 1, 2, 3}
    assert node_lanes(g, plan, 1) == {i: 0 for i in range(len(g.nodes))}
    # a branch chain stays on one lane: a node reading a single-producer
    # intermediate buffer continues its producer's lane (first reader)
    producers = {}
    for i, n in enumerate(g.nodes):
        producers.setdefault(n.y.buf, []).append(i)
    same = sum(1 for i, n in enumerate(g.nodes)
               if len(producers.get(n.x, [])) == 1 and lane[i] == lane[producers[n.x][0]])
    assert same >= 40
    # members of a fused sibling group share their launch's lane
    for u in plan.units:
        idx = [i for i, n in enumerate(g.nodes) if n.kind == "conv" and n in u.members]
        assert len({lane[i] for i in idx}) == 1


def test_schedule_random_sequences_are_race_free():
    rng = random.Random(0)
    for trial in range(200):
        calls = []
        for i in range(rng.randint(1, 40)):
            res = [("r", rng.randint(0, 6)) for _ in range(rng.randint(0, 3))]
            wr = [("r", rng.randint(0, 6)) for _ in range(rng.randint(0, 2))]
            calls.append(Call(None, (), f"c{i}", rng.randint(0, 3), tuple(res), tuple(wr)))
        schedule(calls)
        check_schedule(calls)
        check_schedule(calls, precise=True)


def test_schedule_serialises_accumulating_writers_in_issue_order():
    # three dgrad-like writers of one gradient buffer on three lanes, then its reader
    calls = [Call(None, (), "w0", 1, (), (("d", 5, 0),)), Call(None, (), "w1", 2, (), (("d", 5, 0),)),
             Call(None, (), "w2", 3, (), (("d", 5, 0),)), Call(None, (), "r", 0, (("d", 5, 0),), ())]
    schedule(calls)
    check_schedule(calls)
    check_schedule(calls, precise=True)
    assert calls[1].waits == [1] and calls[2].waits == [2] and calls[3].waits == [3]
    assert calls[1].pwaits == [(1, 0)] and calls[2].pwaits == [(2, 1)] and calls[3].pwaits == [(3, 2)]


def test_schedule_skips_waits_already_implied():
    calls = [Call(None, (), "a", 1, (), (("x",),)), Call(None, (), "b", 0, (("x",),), (("y",),)),
             Call(None, (), "c", 0, (("x",),), (("z",),))]
    schedule(calls)
    assert calls[1].waits == [1] and calls[2].waits == []   # lane 0 already waited for lane 1's tail
    assert calls[1].pwaits == [(1, 0)] and calls[2].pwaits == [] and calls[0].record
    check_schedule(calls)
    check_schedule(calls, precise=True)


def test_producer_waits_do_not_wait_for_later_work():
    # lane 1 issues a (producer) then b (unrelated); lane 0's consumer of a
    # waits for a itself, while the tail wait covers b too
    calls = [Call(None, (), "a", 1, (), (("x",),)), Call(None, (), "b", 1, (), (("y",),)),
             Call(None, (), "c", 0, (("x",),), (("z",),))]
    schedule(calls)
    assert calls[2].waits == [1] and calls[2].pwaits == [(1, 0)]
    assert calls[0].record and not calls[1].record
    check_schedule(calls, precise=True)
