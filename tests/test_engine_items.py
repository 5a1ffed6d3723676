"""CPU: the weight-gradient reduction items the engine records (light_unet/engine.py `_seg`) --
output caps by partial-list length, the wide items of short lists, the launch order (longest
first, `_seg_rounds`) and the exactly-once cover that the fused reduce + AdamW launch requires
(misc.hip reduce_segments_adamw_kernel)."""
import types

from light_unet import engine as E


def _rec(calls):
    """Items recorded by _seg for (src_off, count, istride, tstride, length, dst) calls."""
    me = types.SimpleNamespace(offsets={"a": (0,), "b": (10_000,)}, _items_rec=[])
    for c in calls:
        E.UNetEngine._seg(me, *c)
    return me._items_rec


def test_caps_by_list_length():
    short, mid, long_ = E._SEG_SHORT[0], 384, 1728
    for count, cap in ((short, E._SEG_SHORT[1]), (short + 1, E._SEG_CAPS[0]),
                       (mid, E._SEG_CAPS[1]), (long_, E._SEG_CAPS[2])):
        items = _rec([(0, count, 512, 1, 512, "a")])
        assert all(it[4] <= cap for it in items)
        assert sum(it[4] for it in items) == 512          # every output once
        assert [it[5] for it in items] == sorted(it[5] for it in items)


def test_rounds_and_cover():
    # one long fp32 list (float4 rows) and one short fp64 list
    items = _rec([(0, 1728, 512, 1, 512, "a"), (4096, 4, 3, 12, 16, "b")])
    r = [E._seg_rounds(it) for it in items]
    assert max(r) == E._seg_rounds(items[0])
    # float4 rows of a 32-output item: 8 lanes per row, 32 threads per output, 54 terms, 7 rounds
    it32 = next(it for it in items if it[4] == 32)
    assert E._seg_rounds(it32) == 7
    assert E._items_cover_once(sorted(items, key=lambda it: -E._seg_rounds(it)), 10_016) is False
    only_a = [it for it in items if it[5] < 512]
    assert E._items_cover_once(only_a, 512)
    # an accumulating item disqualifies the fused update
    acc = [list(it) for it in only_a]
    acc[0][6] = 1
    assert not E._items_cover_once(acc, 512)
