"""The rule registry behind the C ABI (match_register, src/main.rs:867) under
a long random sequence of control-plane operations, checked against a Python
dict that restates the reference's semantics:

* add_listening_match (src/main.rs:266-298): a duplicate key answers 0 ("ER")
  and changes nothing; otherwise the rule is inserted and 1 is returned;
* act_on RemoveMatch (src/main.rs:608-625): an unknown key answers 0; only the
  owner may remove (EPERM otherwise);
* EntryChange::Remove (src/main.rs:1058-1069): an endpoint's rules go with it;
* keys are derive(Hash, Eq) on Want: absent Option fields do not take part.

Thousands of keys push the host map through growth, tombstones and reuse.
Registry-only context (USN_HOST_ONLY): no GPU is needed."""
import random

import pytest

from usnetd_amd import lib

NIC = 0
OWNERS = [1, 2, 3, 4, 5]


def canon(w):
    p = w.present & 7
    return (w.dst_addr, w.protocol, p,
            w.dst_port if p & 1 else 0,
            w.src_addr if p & 2 else 0,
            w.src_port if p & 4 else 0)


def rand_want(rng, pool):
    # a small key space so that duplicates, removals and re-adds collide
    w = lib.Want()
    w.dst_addr = 0x0A000000 | rng.randrange(pool)
    w.protocol = rng.choice([6, 17])
    w.present = rng.randrange(8)
    w.dst_port = rng.randrange(1, 64)
    w.src_addr = 0xC0A80000 | rng.randrange(4)
    w.src_port = rng.randrange(1024, 1028)
    if rng.random() < 0.5:   # canonical form: absent fields zero
        if not w.present & 1:
            w.dst_port = 0
        if not w.present & 2:
            w.src_addr = 0
        if not w.present & 4:
            w.src_port = 0
    return w


def make_ctx():
    ctx = lib.Ctx(lib.USN_HOST_ONLY if hasattr(lib, "USN_HOST_ONLY") else -1)
    ctx.endpoint_add(NIC, 0)
    for e in OWNERS:
        ctx.endpoint_add(e, 3, NIC)
    return ctx


@pytest.mark.parametrize("seed,pool,ops", [(1, 64, 6000), (2, 1024, 20000)])
def test_registry_random_ops(seed, pool, ops):
    rng = random.Random(seed)
    ctx = make_ctx()
    model = {}
    alive = set(OWNERS)
    try:
        for step in range(ops):
            op = rng.random()
            w = rand_want(rng, pool)
            k = canon(w)
            if op < 0.55 and alive:
                owner = rng.choice(sorted(alive))
                got = ctx.add_match(w, owner, sticky=rng.random() < 0.2)
                assert got == (0 if k in model else 1), step
                model.setdefault(k, owner)
            elif op < 0.85:
                req = rng.choice(OWNERS)
                if k not in model:
                    assert ctx.remove_match(w, req) == 0, step
                elif model[k] != req:
                    assert ctx.remove_match(w, req) == -1, step   # EPERM
                else:
                    assert ctx.remove_match(w, req) == 1, step
                    del model[k]
            elif op < 0.97:
                assert ctx.lookup(w) == model.get(k, -1), step
            else:   # an endpoint leaves and a new one takes its id
                e = rng.choice(OWNERS)
                if e in alive:
                    ctx.endpoint_remove(e)
                    model = {kk: o for kk, o in model.items() if o != e}
                    alive.discard(e)
                else:
                    ctx.endpoint_add(e, 3, NIC)
                    alive.add(e)
            if step % 997 == 0:
                assert ctx.rule_count() == len(model), step
        assert ctx.rule_count() == len(model)
        got = {canon(w): o for w, o, _ in ctx.rules()}
        assert got == model
    finally:
        ctx.close()


def test_registry_bulk_grow_and_drain():
    """50 000 distinct rules in, every one found, then all removed by their
    owners: the map grows from empty and ends with only tombstones."""
    ctx = make_ctx()
    try:
        ws = []
        for i in range(50000):
            w = lib.make_want(0x0B000000 + i, 6, 80 + (i % 7), src=None, sport=None)
            assert ctx.add_match(w, OWNERS[i % 5]) == 1
            ws.append(w)
        assert ctx.rule_count() == 50000
        for i in range(0, 50000, 97):
            assert ctx.lookup(ws[i]) == OWNERS[i % 5]
        for i, w in enumerate(ws):
            assert ctx.remove_match(w, OWNERS[i % 5]) == 1
        assert ctx.rule_count() == 0
        assert ctx.lookup(ws[0]) == -1
        assert ctx.add_match(ws[0], 1) == 1   # a key can come back after its tombstone
        assert ctx.lookup(ws[0]) == 1
    finally:
        ctx.close()
