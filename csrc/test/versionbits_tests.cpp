// versionbits_tests: the BIP9 threshold state machine and ComputeBlockVersion.
// Parity: reference src/test/versionbits_tests.cpp (a fake CBlockIndex chain mined with chosen
// times/versions, a checker with Period 1000 / Threshold 900 / window [10000, 20000) keyed on
// bit 8, several checkers with partially wiped caches; ComputeBlockVersion walking mainnet's CSV
// deployment through STARTED -> LOCKED_IN -> ACTIVE and the failed/timeout branch).
//
// Instead of the reference's hand-listed transitions, every scenario here is checked against an
// independent period-by-period model of BIP9 (ModelStates), at every height of the fake chain,
// plus randomized chains and randomized cache wiping.
#include "test/unittest.h"

#include "consensus/versionbits.h"
#include "util/strencodings.h"

#include <memory>

using namespace bcp;

namespace {

const int64_t kBegin = 10000, kEnd = 20000;
const int kPeriod = 1000, kThreshold = 900, kBit = 8;

class TestChecker : public AbstractThresholdConditionChecker {
public:
    mutable ThresholdConditionCache cache;
    bool Condition(const CBlockIndex* p, const Consensus::Params&) const override {
        return (p->nVersion & 0xE0000000) == VERSIONBITS_TOP_BITS && (p->nVersion & (1 << kBit)) != 0;
    }
    int64_t BeginTime(const Consensus::Params&) const override { return kBegin; }
    int64_t EndTime(const Consensus::Params&) const override { return kEnd; }
    int Period(const Consensus::Params&) const override { return kPeriod; }
    int Threshold(const Consensus::Params&) const override { return kThreshold; }
    ThresholdState State(const CBlockIndex* prev) const { return GetStateFor(prev, Params().GetConsensus(), cache); }
    int Since(const CBlockIndex* prev) const { return GetStateSinceHeightFor(prev, Params().GetConsensus(), cache); }
};

const int32_t kSignal = VERSIONBITS_TOP_BITS | (1 << kBit);
const int32_t kNoSignal = VERSIONBITS_TOP_BITS;
// a version that has the bit but lacks the top-bits marker: must not count
const int32_t kOldWithBit = 4 | (1 << kBit);

struct FakeChain {
    std::vector<std::unique_ptr<CBlockIndex>> blocks;
    const CBlockIndex* Tip() const { return blocks.empty() ? nullptr : blocks.back().get(); }
    int Height() const { return (int)blocks.size() - 1; }
    // extend up to (but excluding) height `upto` with the given time and version
    FakeChain& Mine(int upto, int64_t time, int32_t version) {
        while ((int)blocks.size() < upto) Add(time, version);
        return *this;
    }
    void Add(int64_t time, int32_t version) {
        auto b = std::make_unique<CBlockIndex>();
        b->nHeight = (int)blocks.size();
        b->pprev = blocks.empty() ? nullptr : blocks.back().get();
        b->nTime = (uint32_t)time;
        b->nVersion = version;
        b->BuildSkip();
        blocks.push_back(std::move(b));
    }
    void Rewind(int height) { blocks.resize(height); }
    const CBlockIndex* At(int h) const { return h < 0 ? nullptr : blocks[h].get(); }
};

// Independent BIP9 model: state of every period present on the chain (period k = heights
// [k*P, (k+1)*P)); period k's state is decided by the median time past of block k*P-1 and the
// signalling count of period k-1.
std::vector<ThresholdState> ModelStates(const FakeChain& c, const TestChecker& chk) {
    const Consensus::Params& p = Params().GetConsensus();
    const int periods = (c.Height() + 1) / kPeriod + 1;
    std::vector<ThresholdState> s(periods, THRESHOLD_DEFINED);
    for (int k = 1; k < periods; k++) {
        const CBlockIndex* boundary = c.At(k * kPeriod - 1);
        const int64_t mtp = boundary->GetMedianTimePast();
        ThresholdState prev = s[k - 1], next = prev;
        if (mtp < kBegin) {
            next = THRESHOLD_DEFINED;
        } else if (prev == THRESHOLD_DEFINED) {
            next = mtp >= kEnd ? THRESHOLD_FAILED : THRESHOLD_STARTED;
        } else if (prev == THRESHOLD_STARTED) {
            if (mtp >= kEnd) {
                next = THRESHOLD_FAILED;
            } else {
                int count = 0;
                for (int h = (k - 1) * kPeriod; h < k * kPeriod; h++) count += chk.Condition(c.At(h), p) ? 1 : 0;
                if (count >= kThreshold) next = THRESHOLD_LOCKED_IN;
            }
        } else if (prev == THRESHOLD_LOCKED_IN) {
            next = THRESHOLD_ACTIVE;
        }
        s[k] = next;
    }
    return s;
}

int ModelSince(const std::vector<ThresholdState>& s, int k) {
    if (s[k] == THRESHOLD_DEFINED) return 0;
    int j = k;
    while (j > 0 && s[j - 1] == s[k]) j--;
    return j * kPeriod;
}

// Compare several checkers (with caches wiped at random) against the model at every height.
// `stride` > 1 samples heights to keep randomized runs fast; period boundaries are always checked.
void CheckAgainstModel(const FakeChain& c, std::vector<TestChecker>& checkers, FastRandomContext& rng, int stride = 1) {
    const std::vector<ThresholdState> model = ModelStates(c, checkers[0]);
    for (size_t i = 0; i < checkers.size(); i++) {
        if (rng.randrange(2)) checkers[i].cache.clear();
    }
    // the block after "prev = nullptr" (genesis) is in period 0
    for (auto& chk : checkers) {
        CHECK_EQ(chk.State(nullptr), THRESHOLD_DEFINED);
        CHECK_EQ(chk.Since(nullptr), 0);
    }
    for (int h = 0; h <= c.Height(); h++) {
        const bool boundary = (h + 2) % kPeriod <= 2;
        if (!boundary && h % stride != 0 && h != c.Height()) continue;
        const int k = (h + 1) / kPeriod; // period of the block after h
        for (auto& chk : checkers) {
            if (rng.randrange(64) == 0) chk.cache.clear();
            const ThresholdState got = chk.State(c.At(h));
            if (got != model[k]) {
                test::RecordFailure(strprintf("height %d: state %s, model %s", h, ThresholdStateName(got),
                                        ThresholdStateName(model[k])),
                              __FILE__, __LINE__);
                return;
            }
            CHECK_EQ(chk.Since(c.At(h)), ModelSince(model, k));
        }
    }
}

ThresholdState StateAtTip(const FakeChain& c, TestChecker& chk) { return chk.State(c.Tip()); }

} // namespace

TEST_CASE(versionbits_tests, scripted_transitions) {
    test::BasicTestingSetup setup("main");
    FastRandomContext rng(true);
    std::vector<TestChecker> chk(4);

    // 1. before the start time nothing happens, whatever is signalled
    FakeChain a;
    a.Mine(1, 1000, kSignal).Mine(3 * kPeriod, 2000, kSignal);
    CHECK_EQ(StateAtTip(a, chk[0]), THRESHOLD_DEFINED);
    CheckAgainstModel(a, chk, rng);

    // 2. start time reached -> STARTED; 899 signals is one short -> stays STARTED
    FakeChain b;
    b.Mine(kPeriod, kBegin - 100, kNoSignal).Mine(2 * kPeriod, kBegin, kNoSignal);
    CHECK_EQ(StateAtTip(b, chk[1]), THRESHOLD_STARTED);
    CHECK_EQ(chk[1].Since(b.Tip()), 2 * kPeriod);
    b.Mine(2 * kPeriod + kThreshold - 1, kBegin + 1, kSignal).Mine(3 * kPeriod, kBegin + 1, kNoSignal);
    CHECK_EQ(StateAtTip(b, chk[1]), THRESHOLD_STARTED);
    CHECK_EQ(chk[1].Since(b.Tip()), 2 * kPeriod);
    // exactly the threshold, interleaved with non-signalling blocks -> LOCKED_IN, then ACTIVE
    for (int i = 0; i < kPeriod; i++) b.Add(kBegin + 2, (i % 10 == 0) ? kNoSignal : kSignal);
    CHECK_EQ(StateAtTip(b, chk[1]), THRESHOLD_LOCKED_IN);
    CHECK_EQ(chk[1].Since(b.Tip()), 4 * kPeriod);
    b.Mine(5 * kPeriod, kBegin + 3, kNoSignal);
    CHECK_EQ(StateAtTip(b, chk[1]), THRESHOLD_ACTIVE);
    CHECK_EQ(chk[1].Since(b.Tip()), 5 * kPeriod);
    // ACTIVE is terminal, even after the timeout
    b.Mine(7 * kPeriod, kEnd + 5000, kNoSignal);
    CHECK_EQ(StateAtTip(b, chk[1]), THRESHOLD_ACTIVE);
    CheckAgainstModel(b, chk, rng);

    // 3. signals without the top-bits marker do not count
    FakeChain c;
    c.Mine(kPeriod, kBegin, kNoSignal).Mine(2 * kPeriod, kBegin, kOldWithBit).Mine(3 * kPeriod, kBegin, kOldWithBit);
    CHECK_EQ(StateAtTip(c, chk[2]), THRESHOLD_STARTED);
    CheckAgainstModel(c, chk, rng);

    // 4. timeout while STARTED -> FAILED (terminal even if everyone signals afterwards)
    FakeChain d;
    d.Mine(kPeriod, kBegin, kNoSignal).Mine(2 * kPeriod, kEnd, kSignal);
    CHECK_EQ(StateAtTip(d, chk[3]), THRESHOLD_FAILED);
    d.Mine(5 * kPeriod, kEnd + 10, kSignal);
    CHECK_EQ(StateAtTip(d, chk[3]), THRESHOLD_FAILED);
    CHECK_EQ(chk[3].Since(d.Tip()), 2 * kPeriod);
    CheckAgainstModel(d, chk, rng);

    // 5. timeout reached during the LOCKED_IN period still activates
    FakeChain e;
    e.Mine(kPeriod, kBegin, kNoSignal).Mine(2 * kPeriod, kBegin + 1, kSignal);
    CHECK_EQ(StateAtTip(e, chk[0]), THRESHOLD_LOCKED_IN);
    e.Mine(3 * kPeriod - 1, kEnd + 1, kNoSignal);
    CHECK_EQ(StateAtTip(e, chk[0]), THRESHOLD_LOCKED_IN);
    e.Mine(3 * kPeriod, kEnd + 2, kNoSignal); // boundary MTP is past the timeout
    CHECK_EQ(StateAtTip(e, chk[0]), THRESHOLD_ACTIVE);
    CheckAgainstModel(e, chk, rng);

    // 6. start and timeout passed within the same period -> straight to FAILED from DEFINED
    FakeChain f;
    f.Mine(kPeriod, kEnd, kSignal).Mine(2 * kPeriod, kEnd, kSignal);
    CHECK_EQ(StateAtTip(f, chk[1]), THRESHOLD_FAILED);
    CheckAgainstModel(f, chk, rng);

    // 7. the median time past, not the block's own time, decides: one late block is not enough
    FakeChain g;
    g.Mine(kPeriod - 1, kBegin - 1, kNoSignal).Mine(kPeriod, kBegin + 5000, kNoSignal);
    CHECK_EQ(StateAtTip(g, chk[2]), THRESHOLD_DEFINED);
    CheckAgainstModel(g, chk, rng);

    // 8. reorg: rewinding and re-mining a different history re-evaluates (caches keyed by block)
    b.Rewind(3 * kPeriod);
    for (auto& k : chk) k.cache.clear();
    b.Mine(4 * kPeriod, kBegin + 2, kNoSignal);
    CHECK_EQ(StateAtTip(b, chk[0]), THRESHOLD_STARTED);
    CheckAgainstModel(b, chk, rng);
}

TEST_CASE(versionbits_tests, randomized_chains_match_model) {
    test::BasicTestingSetup setup("main");
    FastRandomContext rng(true);
    for (int trial = 0; trial < 24; trial++) {
        std::vector<TestChecker> chk(3);
        FakeChain c;
        int64_t t = 5000 + rng.randrange(4000);
        const int periods = 4 + rng.randrange(10);
        for (int k = 0; k < periods; k++) {
            // per period: a time step (times never decrease) and a signalling density near the threshold
            t += rng.randrange(4) == 0 ? 0 : rng.randrange(3500);
            const int density = 850 + rng.randrange(120); // per-mille of signalling blocks
            for (int i = 0; i < kPeriod; i++) {
                const bool sig = (int)rng.randrange(1000) < density;
                const int32_t v = sig ? (rng.randrange(20) == 0 ? kOldWithBit : kSignal | (int32_t)rng.randrange(2))
                                      : kNoSignal | (1 << (kBit + 1));
                c.Add(t + rng.randrange(3), v);
            }
        }
        CheckAgainstModel(c, chk, rng, 97);
        if (test::HasFailures()) break;
    }
}

TEST_CASE(versionbits_tests, statistics) {
    test::BasicTestingSetup setup("main");
    TestChecker chk;
    const Consensus::Params& p = Params().GetConsensus();
    FakeChain c;
    // stats before any block of the second period exists, including inside the very first period
    c.Mine(5, kBegin, kSignal);
    BIP9Stats s = chk.GetStateStatisticsFor(c.Tip(), p);
    CHECK_EQ(s.period, kPeriod);
    CHECK_EQ(s.threshold, kThreshold);
    CHECK_EQ(s.elapsed, 5);
    CHECK_EQ(s.count, 5);
    CHECK(s.possible);
    c.Mine(kPeriod, kBegin, kNoSignal);
    s = chk.GetStateStatisticsFor(c.Tip(), p);
    CHECK_EQ(s.elapsed, 0); // the tip closes a period: stats describe the next (empty) one
    CHECK_EQ(s.count, 0);
    // 100 misses are still recoverable, 101 are not
    c.Mine(kPeriod + 100, kBegin, kNoSignal);
    s = chk.GetStateStatisticsFor(c.Tip(), p);
    CHECK_EQ(s.elapsed, 100);
    CHECK_EQ(s.count, 0);
    CHECK(s.possible);
    c.Add(kBegin, kNoSignal);
    s = chk.GetStateStatisticsFor(c.Tip(), p);
    CHECK(!s.possible);
    c.Mine(kPeriod + 400, kBegin, kSignal);
    s = chk.GetStateStatisticsFor(c.Tip(), p);
    CHECK_EQ(s.elapsed, 400);
    CHECK_EQ(s.count, 299);
}

TEST_CASE(versionbits_tests, deployment_sanity) {
    // every network: bits in range and distinct, masks consistent, windows well formed
    for (const char* chain : {"main", "test", "regtest"}) {
        test::BasicTestingSetup setup(chain);
        const Consensus::Params& p = Params().GetConsensus();
        CHECK(p.nRuleChangeActivationThreshold <= p.nMinerConfirmationWindow);
        CHECK(p.nMinerConfirmationWindow > 0);
        uint32_t seen = 0;
        for (int i = 0; i < (int)Consensus::MAX_VERSION_BITS_DEPLOYMENTS; i++) {
            const auto pos = (Consensus::DeploymentPos)i;
            const Consensus::BIP9Deployment& d = p.vDeployments[i];
            CHECK(d.bit >= 0 && d.bit < VERSIONBITS_NUM_BITS);
            CHECK(d.nStartTime < d.nTimeout);
            const uint32_t mask = VersionBitsMask(p, pos);
            CHECK_EQ(mask, (uint32_t)1 << d.bit);
            CHECK_EQ(mask & (uint32_t)VERSIONBITS_TOP_MASK, 0u);
            // overlapping windows may not share a bit
            for (int j = 0; j < i; j++) {
                const Consensus::BIP9Deployment& o = p.vDeployments[j];
                if (o.bit == d.bit) CHECK(o.nTimeout <= d.nStartTime || d.nTimeout <= o.nStartTime);
            }
            seen |= mask;
            CHECK(VersionBitsDeploymentInfo[i].name != nullptr);
        }
        CHECK(seen != 0);
    }
}

TEST_CASE(versionbits_tests, compute_block_version) {
    // Walk mainnet's CSV deployment: the miner signals its bit while STARTED and LOCKED_IN only.
    test::BasicTestingSetup setup("main");
    const Consensus::Params& p = Params().GetConsensus();
    const auto pos = Consensus::DEPLOYMENT_CSV;
    const int64_t start = p.vDeployments[pos].nStartTime, timeout = p.vDeployments[pos].nTimeout;
    const int period = (int)p.nMinerConfirmationWindow;
    const int threshold = (int)p.nRuleChangeActivationThreshold;
    const uint32_t bit = VersionBitsMask(p, pos);
    // the test-dummy deployment's window is long past on mainnet, so only CSV's bit can show up
    REQUIRE(p.vDeployments[Consensus::DEPLOYMENT_TESTDUMMY].nTimeout < start);

    VersionBitsCache cache;
    FakeChain c;
    auto version = [&]() { return ComputeBlockVersion(c.Tip(), p, cache); };
    // genesis parent: DEFINED -> only the top bits
    CHECK_EQ(version(), VERSIONBITS_TOP_BITS);
    c.Mine(period - 1, start - 1, VERSIONBITS_TOP_BITS);
    CHECK_EQ(version() & (int32_t)bit, 0);
    CHECK_EQ(version() & VERSIONBITS_TOP_MASK, VERSIONBITS_TOP_BITS);
    // a full period with MTP >= start -> STARTED for the next period: signal
    c.Mine(2 * period - 1, start, VERSIONBITS_TOP_BITS);
    CHECK_EQ(version() & (int32_t)bit, 0); // the boundary block is not mined yet
    c.Add(start, VERSIONBITS_TOP_BITS);
    CHECK((version() & (int32_t)bit) != 0);
    CHECK_EQ(VersionBitsState(c.Tip(), p, pos, cache), THRESHOLD_STARTED);
    // a period one short of the threshold keeps it STARTED (still signalling)
    c.Mine(2 * period + threshold - 1, start + 1, VERSIONBITS_TOP_BITS | (int32_t)bit);
    c.Mine(3 * period, start + 1, VERSIONBITS_TOP_BITS);
    CHECK((version() & (int32_t)bit) != 0);
    CHECK_EQ(VersionBitsState(c.Tip(), p, pos, cache), THRESHOLD_STARTED);
    // a full period of signals -> LOCKED_IN (still signalling), then ACTIVE (bit cleared)
    c.Mine(4 * period, start + 2, VERSIONBITS_TOP_BITS | (int32_t)bit);
    CHECK_EQ(VersionBitsState(c.Tip(), p, pos, cache), THRESHOLD_LOCKED_IN);
    CHECK((version() & (int32_t)bit) != 0);
    CHECK_EQ(VersionBitsStateSinceHeight(c.Tip(), p, pos, cache), 4 * period);
    c.Mine(5 * period, start + 3, VERSIONBITS_TOP_BITS);
    CHECK_EQ(VersionBitsState(c.Tip(), p, pos, cache), THRESHOLD_ACTIVE);
    CHECK_EQ(version() & (int32_t)bit, 0);
    CHECK_EQ(version(), VERSIONBITS_TOP_BITS);

    // the failure branch: started but never locked in before the timeout -> FAILED, bit cleared
    VersionBitsCache cache2;
    FakeChain f;
    f.Mine(period, start, VERSIONBITS_TOP_BITS).Mine(2 * period, start, VERSIONBITS_TOP_BITS);
    CHECK((ComputeBlockVersion(f.Tip(), p, cache2) & (int32_t)bit) != 0);
    f.Mine(3 * period, timeout, VERSIONBITS_TOP_BITS);
    CHECK_EQ(VersionBitsState(f.Tip(), p, pos, cache2), THRESHOLD_FAILED);
    CHECK_EQ(ComputeBlockVersion(f.Tip(), p, cache2), VERSIONBITS_TOP_BITS);
}
