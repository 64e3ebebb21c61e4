// shardplan_tests: the GPU verify service's device-aware shard plan (node/gpuverify.h
// PlanShards), pure CPU. Replaces the reference's CCheckQueue split of a block's checks across
// -par threads (src/checkqueue.h:27-164): here a batch is spread over distinct GPUs first, and a
// second lane on one GPU takes a shard only for very large batches.
#include "test/unittest.h"

#include "node/gpuverify.h"

#include <set>

using namespace bcp;

namespace {

std::vector<int> DefaultLanes(int ndev) { // every device, twice, round-robin
    std::vector<int> l;
    for (int rep = 0; rep < 2; rep++)
        for (int d = 0; d < ndev; d++) l.push_back(d);
    return l;
}

// the plan covers [0, n) contiguously, in order, with no empty shard and no lane twice
void CheckCover(const std::vector<VerifyShard>& plan, size_t n, size_t nlanes) {
    size_t lo = 0;
    std::set<size_t> used;
    for (const auto& s : plan) {
        CHECK_EQ(s.lo, lo);
        CHECK(s.hi > s.lo);
        CHECK(s.lane < nlanes);
        CHECK(used.insert(s.lane).second);
        lo = s.hi;
    }
    CHECK_EQ(lo, n);
}

std::set<int> DevicesOf(const std::vector<VerifyShard>& plan, const std::vector<int>& lanes) {
    std::set<int> d;
    for (const auto& s : plan) d.insert(lanes[s.lane]);
    return d;
}

} // namespace

TEST_CASE(shardplan_tests, ecdsa_one_two_eight_devices) {
    const size_t MINDEV = 4096, MINLANE = 65536; // the service's ECDSA defaults
    // 1 device, lanes [0, 0]
    {
        const auto L = DefaultLanes(1);
        auto p = PlanShards(512, L, MINDEV, MINLANE);
        CheckCover(p, 512, L.size());
        CHECK_EQ(p.size(), (size_t)1);
        p = PlanShards(42000, L, MINDEV, MINLANE);
        CheckCover(p, 42000, L.size());
        CHECK_EQ(p.size(), (size_t)1); // a second lane on one GPU does not pay at 42k
        p = PlanShards(199000, L, MINDEV, MINLANE);
        CheckCover(p, 199000, L.size());
        CHECK_EQ(p.size(), (size_t)2); // the 199k worst case takes both lanes
        CHECK_EQ(DevicesOf(p, L).size(), (size_t)1);
    }
    // 2 devices, lanes [0, 1, 0, 1]
    {
        const auto L = DefaultLanes(2);
        auto p = PlanShards(512, L, MINDEV, MINLANE);
        CheckCover(p, 512, L.size());
        CHECK_EQ(p.size(), (size_t)1);
        p = PlanShards(42000, L, MINDEV, MINLANE);
        CheckCover(p, 42000, L.size());
        CHECK_EQ(p.size(), (size_t)2);
        CHECK_EQ(DevicesOf(p, L).size(), (size_t)2);
        p = PlanShards(199000, L, MINDEV, MINLANE);
        CheckCover(p, 199000, L.size());
        CHECK_EQ(p.size(), (size_t)2); // 99.5k per device: still one lane each
        CHECK_EQ(DevicesOf(p, L).size(), (size_t)2);
        p = PlanShards(300000, L, MINDEV, MINLANE); // 150k per device: both lanes of both
        CheckCover(p, 300000, L.size());
        CHECK_EQ(p.size(), (size_t)4);
    }
    // 8 devices, lanes [0..7, 0..7]
    {
        const auto L = DefaultLanes(8);
        auto p = PlanShards(512, L, MINDEV, MINLANE);
        CheckCover(p, 512, L.size());
        CHECK_EQ(p.size(), (size_t)1);
        p = PlanShards(42000, L, MINDEV, MINLANE); // an 8 MB P2PKH block: all 8 GPUs
        CheckCover(p, 42000, L.size());
        CHECK_EQ(p.size(), (size_t)8);
        CHECK_EQ(DevicesOf(p, L).size(), (size_t)8);
        for (const auto& s : p) CHECK(s.hi - s.lo == 5250);
        p = PlanShards(199000, L, MINDEV, MINLANE);
        CheckCover(p, 199000, L.size());
        CHECK_EQ(p.size(), (size_t)8);
        CHECK_EQ(DevicesOf(p, L).size(), (size_t)8);
        p = PlanShards(20000, L, MINDEV, MINLANE); // 20000 / 4096 = 4 devices
        CheckCover(p, 20000, L.size());
        CHECK_EQ(p.size(), (size_t)4);
        CHECK_EQ(DevicesOf(p, L).size(), (size_t)4);
    }
}

TEST_CASE(shardplan_tests, duplicate_lane_lists_and_edges) {
    // the test suites' one-GPU sharding ([0, 0, 0, 0] with small floors) keeps working
    const std::vector<int> L4 = {0, 0, 0, 0};
    auto p = PlanShards(10000, L4, 1, 1024);
    CheckCover(p, 10000, L4.size());
    CHECK_EQ(p.size(), (size_t)4);
    p = PlanShards(3000, L4, 1, 1024);
    CheckCover(p, 3000, L4.size());
    CHECK_EQ(p.size(), (size_t)2);
    CHECK(PlanShards(0, L4, 1, 1).empty());
    CHECK(PlanShards(10, {}, 1, 1).empty());
    p = PlanShards(7, {3, 5}, 1, 1); // odd split: 4 + 3
    CheckCover(p, 7, 2);
    CHECK_EQ(p.size(), (size_t)2);
    CHECK_EQ(p[0].hi - p[0].lo, (size_t)4);
    // an explicit list [2, 2, 5]: devices 2 and 5 first; device 2's second lane only when large
    const std::vector<int> L3 = {2, 2, 5};
    p = PlanShards(10000, L3, 4096, 65536);
    CheckCover(p, 10000, L3.size());
    CHECK_EQ(p.size(), (size_t)2);
    CHECK_EQ(p[0].lane, (size_t)0);
    CHECK_EQ(p[1].lane, (size_t)2);
    p = PlanShards(400000, L3, 4096, 65536);
    CheckCover(p, 400000, L3.size());
    CHECK_EQ(p.size(), (size_t)3);
}
