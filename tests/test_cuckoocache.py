"""Signature/script cache behaviour (reference src/test/cuckoocache_tests.cpp): hit rate
across loads, erased entries are overwritten first, and a sliding window of blocks keeps
its fresh entries (generations)."""
import pytest

native = pytest.importorskip("bitcoincashplus_amd._bcpnative")


@pytest.mark.parametrize("load", [0.1, 0.2, 0.4, 0.8, 1.6])
def test_hit_rate(load):
    hits = native.cuckoo_hit_rate(32, load)
    assert hits * max(load, 1.0) > 0.98


def test_erase_prefers_erased_slots():
    erased, stale, fresh = native.cuckoo_erase(32)
    assert fresh > 0.999
    assert stale > 2 * erased


def test_generations_keep_recent_entries():
    min_hit, out_of_tight = native.cuckoo_generations(32, 10.0)
    assert min_hit > 0.99
    assert out_of_tight < 0.01
