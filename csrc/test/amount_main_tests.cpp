// amount_tests: Amount arithmetic and CFeeRate (GetFee truncation, the +-1 satoshi floor for a
// non-zero rate, the fee/size constructor's per-kB resolution, no overflow at the largest size).
// main_tests: block subsidy halvings under main, regtest (150) and another interval, and the
// 21M limit of the summed subsidy.
// Parity: reference src/test/amount_tests.cpp (AmountTests, GetFeeTest) and
// src/test/main_tests.cpp (block_subsidy_test, subsidy_limit_test; test_combiner_all tests a
// boost::signals2 combiner this code base does not have).
#include "test/unittest.h"

#include "consensus/params.h"
#include "primitives/amount.h"

#include <limits>

using namespace bcp;
using bcp::test::BasicTestingSetup;

TEST_CASE(amount_tests, AmountTests) {
    CHECK(Amount(2) <= Amount(2));
    CHECK(Amount(2) <= Amount(3));
    CHECK(Amount(3) >= Amount(2));
    CHECK(Amount(-1) < Amount(0));
    CHECK(Amount(0) > Amount(-1));
    CHECK(Amount(0) != Amount(1));
    Amount amount = 0;
    CHECK_EQ(amount += 1, Amount(1));
    CHECK_EQ(amount += -1, Amount(0));
    CHECK_EQ(amount -= 1, Amount(-1));
    CHECK_EQ(amount -= -1, Amount(0));
    CHECK_EQ(COIN + COIN, Amount(2 * COIN));
    CHECK_EQ(2 * COIN + COIN, Amount(3 * COIN));
    CHECK_EQ(-1 * COIN + COIN, Amount(0));
    CHECK_EQ(COIN - 2 * COIN, -1 * COIN);
    CHECK_EQ(10 * Amount(10), Amount(100));
    CHECK_EQ(Amount(10) / 3, Amount(3));
    CHECK_EQ((double)(10 * COIN) / COIN, 10.0);
    CHECK_EQ(Amount(10) / -3, Amount(-3));
    CHECK_EQ(Amount(101) / 3, Amount(33));
    CHECK_EQ(Amount(100) % 3, Amount(1));
    CHECK_EQ(Amount(101) % 3, Amount(2));
}

TEST_CASE(amount_tests, GetFeeTest) {
    CFeeRate feeRate(0);
    CHECK_EQ(feeRate.GetFee(0), Amount(0));
    CHECK_EQ(feeRate.GetFee(100000), Amount(0));

    feeRate = CFeeRate(1000); // returns the size
    for (size_t n : {0, 1, 121, 999, 1000, 9000}) CHECK_EQ(feeRate.GetFee(n), (Amount)n);
    feeRate = CFeeRate(-1000);
    for (size_t n : {0, 1, 121, 999, 1000, 9000}) CHECK_EQ(feeRate.GetFee(n), -(Amount)n);

    feeRate = CFeeRate(123); // truncates, but never to 0 for a non-zero size
    CHECK_EQ(feeRate.GetFee(0), Amount(0));
    CHECK_EQ(feeRate.GetFee(8), Amount(1));
    CHECK_EQ(feeRate.GetFee(9), Amount(1));
    CHECK_EQ(feeRate.GetFee(121), Amount(14));
    CHECK_EQ(feeRate.GetFee(122), Amount(15));
    CHECK_EQ(feeRate.GetFee(999), Amount(122));
    CHECK_EQ(feeRate.GetFee(1000), Amount(123));
    CHECK_EQ(feeRate.GetFee(9000), Amount(1107));
    feeRate = CFeeRate(-123);
    CHECK_EQ(feeRate.GetFee(0), Amount(0));
    CHECK_EQ(feeRate.GetFee(8), Amount(-1));
    CHECK_EQ(feeRate.GetFee(9), Amount(-1));

    CHECK(CFeeRate(-1, 1000) == CFeeRate(-1));
    CHECK(CFeeRate(0, 1000) == CFeeRate(0));
    CHECK(CFeeRate(1, 1000) == CFeeRate(1));
    CHECK(CFeeRate(1, 1001) == CFeeRate(0)); // satoshis per kB resolution
    CHECK(CFeeRate(2, 1001) == CFeeRate(1));
    CHECK(CFeeRate(26, 789) == CFeeRate(32));
    CHECK(CFeeRate(27, 789) == CFeeRate(34));
    (void)CFeeRate(MAX_MONEY, std::numeric_limits<size_t>::max() >> 1).GetFeePerK(); // no overflow trap
}

namespace {

void TestBlockSubsidyHalvings(const Consensus::Params& params) {
    const int maxHalvings = 64;
    const Amount nInitialSubsidy = 50 * COIN;
    Amount nPrevious = 2 * nInitialSubsidy;
    for (int nHalvings = 0; nHalvings < maxHalvings; nHalvings++) {
        const Amount nSubsidy = GetBlockSubsidy(nHalvings * params.nSubsidyHalvingInterval, params);
        CHECK(nSubsidy <= nInitialSubsidy);
        CHECK_EQ(nSubsidy, nPrevious / 2);
        nPrevious = nSubsidy;
    }
    CHECK_EQ(GetBlockSubsidy(maxHalvings * params.nSubsidyHalvingInterval, params), Amount(0));
}

void TestBlockSubsidyHalvings(int interval) {
    Consensus::Params p;
    p.nSubsidyHalvingInterval = interval;
    TestBlockSubsidyHalvings(p);
}

} // namespace

TEST_CASE(main_tests, block_subsidy_test) {
    BasicTestingSetup setup("main");
    TestBlockSubsidyHalvings(Params().GetConsensus()); // as in main
    TestBlockSubsidyHalvings(150);                     // as in regtest
    TestBlockSubsidyHalvings(1000);
}

TEST_CASE(main_tests, subsidy_limit_test) {
    BasicTestingSetup setup("main");
    const Consensus::Params& params = Params().GetConsensus();
    Amount nSum = 0;
    for (int nHeight = 0; nHeight < 14000000; nHeight += 1000) {
        const Amount nSubsidy = GetBlockSubsidy(nHeight, params);
        CHECK(nSubsidy <= 50 * COIN);
        nSum += 1000 * nSubsidy;
        CHECK(MoneyRange(nSum));
    }
    CHECK_EQ(nSum, Amount(2099999997690000LL));
}
