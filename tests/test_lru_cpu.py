"""Host logic of the resident-table LRU (horreum_amd/table.py _ResidentLRU,
ADVICE r3): byte accounting when a table is collected without release(),
when a dead table's id is reused, and when a table moves between engines.
No GPU: fake tables and engines stand in."""
import gc

from horreum_amd import table as tbl


class _Eng:
    pass


class _Tab:
    def __init__(self):
        self._resident = None


def test_collected_table_leaves_the_lru():
    lru = tbl._ResidentLRU(1000)
    t = _Tab()
    lru.touch(t, 300)
    assert lru.total == 300
    del t
    gc.collect()
    assert lru.total == 0 and not lru.items


def test_reused_id_is_counted_and_evictable():
    """An entry whose weakref is dead under a live table's id (the id was
    reused before the callback ran) is replaced, not merely moved: the new
    table is counted and can be evicted."""
    import weakref
    eng = _Eng()
    lru = tbl._lru(eng)
    lru.budget = 1000
    gone = _Tab()
    dead = weakref.ref(gone)
    del gone
    gc.collect()
    b = _Tab()
    b._resident = (eng, object())
    lru.items[id(b)] = (dead, 600)
    lru.total = 600
    lru.touch(b, 500)
    assert lru.total == 500 and lru.items[id(b)][0]() is b
    c = _Tab()
    c._resident = (eng, object())
    lru.touch(c, 700)  # over budget: b evicted, its resident state cleared
    assert b._resident is None and c._resident is not None
    assert lru.total == 700


def test_engine_switch_keeps_the_new_engines_state():
    e1, e2 = _Eng(), _Eng()
    l1, l2 = tbl._lru(e1), tbl._lru(e2)
    l1.budget = l2.budget = 1000
    t = _Tab()
    t._resident = (e1, object())
    l1.touch(t, 400)
    # the table moved to e2 (SSTable.resident drops it from e1's LRU first;
    # here it is left behind to check that e1's eviction spares e2's state)
    t._resident = (e2, object())
    l2.touch(t, 400)
    other = _Tab()
    other._resident = (e1, object())
    l1.touch(other, 900)  # e1 evicts its stale entry for t
    assert t._resident is not None and t._resident[0] is e2
    l2.drop(t)
    assert l2.total == 0
