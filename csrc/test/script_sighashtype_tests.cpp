// script_sighashtype_tests: the SigHashType wrapper (csrc/script/sighashtype.h).
// Parity: reference src/test/script_sighashtype_tests.cpp (base type extraction, the FORKID
// and ANYONECANPAY flags, the copy-and-modify setters and their raw values).
#include "test/unittest.h"

#include "script/sighashtype.h"

using namespace bcp;

TEST_CASE(script_sighashtype_tests, base_types_and_flags) {
    CHECK(SigHashType().getBaseSigHashType() == BaseSigHashType::ALL);
    CHECK(SigHashType(SIGHASH_ALL).getBaseSigHashType() == BaseSigHashType::ALL);
    CHECK(SigHashType(SIGHASH_NONE).getBaseSigHashType() == BaseSigHashType::NONE);
    CHECK(SigHashType(SIGHASH_SINGLE).getBaseSigHashType() == BaseSigHashType::SINGLE);
    CHECK(SigHashType(SIGHASH_ALL | SIGHASH_FORKID).hasForkId());
    CHECK(!SigHashType(SIGHASH_ALL | SIGHASH_FORKID).hasAnyoneCanPay());
    CHECK(!SigHashType(SIGHASH_ALL | SIGHASH_ANYONECANPAY).hasForkId());
    CHECK(SigHashType(SIGHASH_ALL | SIGHASH_ANYONECANPAY).hasAnyoneCanPay());
    for (BaseSigHashType b : {BaseSigHashType::ALL, BaseSigHashType::NONE, BaseSigHashType::SINGLE})
        CHECK(SigHashType().withBaseSigHash(b).getBaseSigHashType() == b);
    CHECK(SigHashType().withForkId(true).hasForkId());
    CHECK(SigHashType().withAnyoneCanPay(true).hasAnyoneCanPay());
    // a raw value without a base type is refused
    for (uint32_t bad : {0u, 4u, 0x40u, 0x1fu}) {
        bool threw = false;
        try {
            SigHashType t(bad);
            (void)t;
        } catch (const std::runtime_error&) {
            threw = true;
        }
        CHECK(threw);
    }
}

TEST_CASE(script_sighashtype_tests, raw_values) {
    const SigHashType all = SigHashType().withBaseSigHash(BaseSigHashType::ALL);
    const SigHashType none = SigHashType().withBaseSigHash(BaseSigHashType::NONE);
    const SigHashType single = SigHashType().withBaseSigHash(BaseSigHashType::SINGLE);
    CHECK_EQ(all.withForkId(true).getRawSigHashType(), (uint32_t)(SIGHASH_ALL | SIGHASH_FORKID));
    CHECK_EQ(none.withForkId(true).getRawSigHashType(), (uint32_t)(SIGHASH_NONE | SIGHASH_FORKID));
    CHECK_EQ(single.withForkId(true).getRawSigHashType(), (uint32_t)(SIGHASH_SINGLE | SIGHASH_FORKID));
    CHECK_EQ(all.withAnyoneCanPay(true).getRawSigHashType(), (uint32_t)(SIGHASH_ALL | SIGHASH_ANYONECANPAY));
    CHECK_EQ(none.withAnyoneCanPay(true).getRawSigHashType(), (uint32_t)(SIGHASH_NONE | SIGHASH_ANYONECANPAY));
    CHECK_EQ(single.withAnyoneCanPay(true).getRawSigHashType(), (uint32_t)(SIGHASH_SINGLE | SIGHASH_ANYONECANPAY));
    CHECK_EQ(all.withAnyoneCanPay(true).withForkId(true).getRawSigHashType(),
             (uint32_t)(SIGHASH_ALL | SIGHASH_ANYONECANPAY | SIGHASH_FORKID));
    // setters replace, in either order
    CHECK(!all.withForkId(true).withForkId(false).hasForkId());
    CHECK(all.withForkId(false).withForkId(true).hasForkId());
    CHECK(!all.withAnyoneCanPay(true).withAnyoneCanPay(false).hasAnyoneCanPay());
    CHECK(all.withAnyoneCanPay(false).withAnyoneCanPay(true).hasAnyoneCanPay());
    // changing the base keeps the flags
    const SigHashType t = all.withAnyoneCanPay(true).withForkId(true).withBaseSigHash(BaseSigHashType::NONE);
    CHECK(t.getBaseSigHashType() == BaseSigHashType::NONE);
    CHECK(t.hasForkId() && t.hasAnyoneCanPay());
}
