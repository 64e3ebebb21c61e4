// Small reference unit suites in one file:
// * dstencode_tests: the same key and script hash encode to the reference's cashaddr
//   ("bitcoincashplus:" prefix) and base58 mainnet strings, and both forms decode back;
// * base32_tests: RFC 4648 vectors (the Tor onion encoding);
// * bswap_tests: 16/32/64-bit byte swaps;
// * random_tests: deterministic FastRandomContexts agree, seeded ones differ, randbits/randrange
//   stay in range; the OS RNG start-up check;
// * sanity_tests: the start-up ECC check (libc/libstdc++/libsodium checks have no counterpart:
//   this build uses neither glibc back-compat shims nor libsodium).
// Parity: reference src/test/{dstencode,base32,bswap,random,sanity}_tests.cpp.
#include "test/unittest.h"

#include "keys/key.h"
#include "util/strencodings.h"

#include <cstdint>

using namespace bcp;
using bcp::test::BasicTestingSetup;

TEST_CASE(dstencode_tests, test_addresses) {
    BasicTestingSetup setup("main");
    const std::vector<unsigned char> hash = {0, 17, 128, 5, 246, 174, 201, 130, 217, 236,
                                             131, 136, 199, 148, 26, 202, 163, 58, 140, 221};
    uint160 h;
    memcpy(h.begin(), hash.data(), 20);
    const CTxDestination dstKey = CKeyID(h);
    const CTxDestination dstScript = CScriptID(h);
    const std::string cashaddr_pubkey = "bitcoincashplus:qqqprqq976hvnqkeajpc33u5rt92xw5vm5ylgfku0f";
    const std::string cashaddr_script = "bitcoincashplus:pqqprqq976hvnqkeajpc33u5rt92xw5vm5n64x3l55";
    const std::string base58_pubkey = "CGUFXy9eQgs3eunVAEqFdS9tnkEcgLw9VD";
    const std::string base58_script = "AFnEcRfCrnYfZk6439AfConxeDwu6kYGdb";
    const CChainParams& params = Params();
    const bool was = UseCashAddr();
    SetUseCashAddr(true);
    CHECK_EQ(EncodeDestination(dstKey, params), cashaddr_pubkey);
    CHECK_EQ(EncodeDestination(dstScript, params), cashaddr_script);
    SetUseCashAddr(false);
    CHECK_EQ(EncodeDestination(dstKey, params), base58_pubkey);
    CHECK_EQ(EncodeDestination(dstScript, params), base58_script);
    SetUseCashAddr(was);
    CHECK(DecodeDestination(cashaddr_pubkey, params) == dstKey);
    CHECK(DecodeDestination(cashaddr_script, params) == dstScript);
    CHECK(DecodeDestination(base58_pubkey, params) == dstKey);
    CHECK(DecodeDestination(base58_script, params) == dstScript);
    for (const std::string& s : {cashaddr_pubkey, cashaddr_script, base58_pubkey, base58_script})
        CHECK(IsValidDestinationString(s, params));
    CHECK(!IsValidDestinationString("notvalid", params));
}

TEST_CASE(base32_tests, base32_testvectors) {
    const char* in[] = {"", "f", "fo", "foo", "foob", "fooba", "foobar"};
    const char* out[] = {"", "my======", "mzxq====", "mzxw6===", "mzxw6yq=", "mzxw6ytb", "mzxw6ytboi======"};
    for (int i = 0; i < 7; i++) {
        const std::string s(in[i]);
        CHECK_EQ(EncodeBase32(reinterpret_cast<const unsigned char*>(s.data()), s.size()), std::string(out[i]));
        bool invalid = false;
        const std::vector<unsigned char> dec = DecodeBase32(out[i], &invalid);
        CHECK(!invalid);
        CHECK_EQ(std::string(dec.begin(), dec.end()), s);
    }
}

TEST_CASE(bswap_tests, bswap_tests) {
    CHECK_EQ(__builtin_bswap16((uint16_t)0x1234), (uint16_t)0x3412);
    CHECK_EQ(__builtin_bswap32(0x56789abcu), 0xbc9a7856u);
    CHECK_EQ(__builtin_bswap64(0xdef0123456789abcull), 0xbc9a78563412f0deull);
}

TEST_CASE(random_tests, osrandom_tests) { CHECK(Random_SanityCheck()); }

TEST_CASE(random_tests, fastrandom_tests) {
    FastRandomContext ctx1(true), ctx2(true);
    CHECK_EQ(ctx1.rand32(), ctx2.rand32());
    CHECK_EQ(ctx1.rand32(), ctx2.rand32());
    CHECK_EQ(ctx1.rand64(), ctx2.rand64());
    CHECK_EQ(ctx1.randbits(3), ctx2.randbits(3));
    CHECK_EQ(ctx1.randbits(7), ctx2.randbits(7));
    CHECK_EQ(ctx1.rand32(), ctx2.rand32());
    CHECK_EQ(ctx1.randbits(3), ctx2.randbits(3));
    FastRandomContext ctx3, ctx4;
    CHECK(ctx3.rand64() != ctx4.rand64()); // 2^-64
}

TEST_CASE(random_tests, fastrandom_randbits) {
    FastRandomContext ctx1, ctx2;
    for (int bits = 0; bits < 63; ++bits) {
        for (int j = 0; j < 1000; ++j) {
            const uint64_t rangebits = ctx1.randbits(bits);
            CHECK_EQ(rangebits >> bits, (uint64_t)0);
            const uint64_t range = (uint64_t(1) << bits) | rangebits;
            CHECK(ctx2.randrange(range) < range);
        }
    }
}

TEST_CASE(sanity_tests, basic_sanity) { CHECK(ECC_InitSanityCheck()); }

// Parity: reference src/test/base64_tests.cpp (base64_testvectors, RFC 4648).
TEST_CASE(base64_tests, base64_testvectors) {
    const char* in[] = {"", "f", "fo", "foo", "foob", "fooba", "foobar"};
    const char* out[] = {"", "Zg==", "Zm8=", "Zm9v", "Zm9vYg==", "Zm9vYmE=", "Zm9vYmFy"};
    for (int i = 0; i < 7; i++) {
        CHECK_EQ(EncodeBase64(std::string(in[i])), std::string(out[i]));
        bool invalid = false;
        const std::vector<unsigned char> dec = DecodeBase64(out[i], &invalid);
        CHECK(!invalid);
        CHECK_EQ(std::string(dec.begin(), dec.end()), std::string(in[i]));
    }
}
