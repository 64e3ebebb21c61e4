"""Container utilities (reference src/test/limitedmap_tests.cpp, indirectmap usage in the
mempool, memusage.h): bounded eviction by smallest value, value updates, dereferencing keys,
allocator-rounded heap accounting."""
import pytest

native = pytest.importorskip("bitcoincashplus_amd._bcpnative")


def test_limitedmap_evicts_smallest_values():
    m = native.LimitedMap(10)
    for i in range(10):
        m.insert(i, i + 100)  # values 100..109
    assert len(m) == 10 and m.get(0) == 100
    m.insert(20, 500)  # full: the smallest value (key 0 -> 100) goes
    assert len(m) == 10 and m.get(0) is None and m.get(20) == 500
    m.update(1, 50)  # key 1 now holds the smallest value
    m.insert(21, 600)
    assert m.get(1) is None and m.get(2) == 102
    m.insert(2, 999)  # existing key: no change, no eviction
    assert m.get(2) == 102 and len(m) == 10
    m.erase(2)
    assert m.get(2) is None and len(m) == 9
    m.set_max_size(5)  # shrinking drops the smallest values
    assert len(m) == 5 and sorted(m.keys()) == [7, 8, 9, 20, 21]


def test_indirectmap_orders_by_pointee():
    order, found, count = native.indirectmap_probe([30, 10, 20, 5])
    assert order == [5, 10, 20, 30]
    assert found == 0 and count == 1


def test_malloc_usage_model():
    assert native.malloc_usage(0) == 0
    assert native.malloc_usage(1) == 32
    assert native.malloc_usage(24) == 32
    assert native.malloc_usage(25) == 48
    assert native.memusage_vector_u8(100) == native.malloc_usage(100)
