// RPC argument handling, raw-transaction signing, amounts, JSON parsing and CLI conversion,
// through the real command table against an in-memory regtest node.
// Parity: reference src/test/rpc_tests.cpp (rpc_rawparams, rpc_rawsign,
// rpc_rawsign_missing_amount, rpc_createraw_op_return, rpc_format_monetary_values,
// rpc_parse_monetary_values, json_parse_errors, rpc_convert_values_generatetoaddress). The
// signing cases use keys and a multisig made here; amounts are checked over generated values.
#include "keys/key.h"
#include "rpc/server.h"
#include "script/standard.h"
#include "test/unittest.h"
#include "util/strencodings.h"

#include <mutex>

namespace bcp {
namespace {

// "method arg1 arg2 ..." through the CLI converter and the command table; an RPC error becomes
// a std::runtime_error carrying its message
UniValue Call(const std::string& line) {
    static std::once_flag once;
    std::call_once(once, [] {
        RegisterAllRPCCommands(tableRPC);
        SetRPCWarmupFinished();
    });
    std::vector<std::string> words;
    for (const std::string& w : SplitString(line, ' '))
        if (!w.empty()) words.push_back(w);
    JSONRPCRequest req;
    req.strMethod = words[0];
    req.params = RPCConvertValues(req.strMethod, std::vector<std::string>(words.begin() + 1, words.end()));
    try {
        return tableRPC.execute(req);
    } catch (const JSONRPCException& e) {
        throw std::runtime_error(find_value(e.obj, "message").get_str());
    }
}

bool Fails(const std::string& line) {
    try {
        Call(line);
    } catch (const std::runtime_error&) {
        return true;
    }
    return false;
}

UniValue Num(const std::string& s) {
    UniValue v;
    v.setNumStr(s);
    return v;
}

const std::string TXID = std::string(62, '0') + "2a";

} // namespace

TEST_CASE(rpc_tests, raw_transaction_arguments) {
    test::TestingSetup setup("regtest");
    // wrong arity and types
    for (const char* bad : {"getrawtransaction", "getrawtransaction zz", "createrawtransaction",
                            "createrawtransaction null null", "createrawtransaction not_an_array",
                            "createrawtransaction [] []", "createrawtransaction {} {}",
                            "createrawtransaction [] {} surplus", "decoderawtransaction",
                            "decoderawtransaction null", "decoderawtransaction 0badc0de", "signrawtransaction",
                            "signrawtransaction null", "signrawtransaction 00ff", "sendrawtransaction",
                            "sendrawtransaction null", "sendrawtransaction 0badc0de"})
        CHECK(Fails(bad));
    CHECK(!Fails("createrawtransaction [] {}"));
    // a transaction built here decodes to what was put in
    CKey k;
    k.MakeNewKey(true);
    const std::string addr = EncodeDestination(k.GetPubKey().GetID(), Params());
    const std::string raw =
        Call("createrawtransaction [{\"txid\":\"" + TXID + "\",\"vout\":3}] {\"" + addr + "\":1.25} 77").get_str();
    UniValue d = Call("decoderawtransaction " + raw);
    CHECK_EQ(find_value(d, "version").get_int(), 2);
    CHECK_EQ(find_value(d, "locktime").get_int(), 77);
    CHECK_EQ(find_value(d, "size").get_int(), (int)(raw.size() / 2));
    CHECK_EQ(find_value(find_value(d, "vin")[0], "vout").get_int(), 3);
    CHECK_EQ(find_value(find_value(d, "vout")[0], "value").getValStr(), std::string("1.25000000"));
    CHECK(Fails("decoderawtransaction " + raw + " surplus"));
    CHECK(Fails("sendrawtransaction " + raw + " false surplus"));
    // signing options
    CHECK(!Fails("signrawtransaction " + raw));
    CHECK(!Fails("signrawtransaction " + raw + " null null ALL|FORKID|ANYONECANPAY"));
    CHECK(!Fails("signrawtransaction " + raw + " [] [] SINGLE|FORKID"));
    CHECK(Fails("signrawtransaction " + raw + " null null NOT_A_SIGHASH"));
    // bad inputs to createrawtransaction
    CHECK(Fails("createrawtransaction [{\"txid\":\"zz\",\"vout\":0}] {}"));
    CHECK(Fails("createrawtransaction [{\"txid\":\"" + TXID + "\",\"vout\":-1}] {}"));
    CHECK(Fails("createrawtransaction [{\"txid\":\"" + TXID + "\"}] {}"));
    CHECK(Fails("createrawtransaction [] {\"" + addr + "\":1,\"" + addr + "\":2}")); // duplicate address
    CHECK(Fails("createrawtransaction [] {\"" + addr + "\":-1}"));
}

TEST_CASE(rpc_tests, sign_multisig_and_missing_amount) {
    test::TestingSetup setup("regtest");
    CKey k1, k2;
    k1.MakeNewKey(true);
    k2.MakeNewKey(true);
    const CScript redeem = GetScriptForMultisig(1, {k1.GetPubKey(), k2.GetPubKey()});
    const CScript p2sh = GetScriptForDestination(CScriptID(redeem));
    const std::string prev = "[{\"txid\":\"" + TXID + "\",\"vout\":1,\"scriptPubKey\":\"" + HexStr(p2sh) +
                             "\",\"redeemScript\":\"" + HexStr(redeem) + "\"";
    const std::string withAmount = prev + ",\"amount\":2.5}]";
    const std::string noAmount = prev + "}]";
    const std::string to = EncodeDestination(CScriptID(redeem), Params());
    const std::string raw = Call("createrawtransaction " + withAmount + " {\"" + to + "\":2.4}").get_str();
    const std::string key1 = "\"" + EncodeSecret(k1, Params()) + "\"", key2 = "\"" + EncodeSecret(k2, Params()) + "\"";
    // no keys: incomplete; either key completes a 1-of-2
    CHECK(!find_value(Call("signrawtransaction " + raw + " " + withAmount + " []"), "complete").get_bool());
    CHECK(find_value(Call("signrawtransaction " + raw + " " + withAmount + " [" + key2 + "]"), "complete").get_bool());
    CHECK(find_value(Call("signrawtransaction " + raw + " " + withAmount + " [" + key1 + "," + key2 + "]"), "complete")
              .get_bool());
    // a replay-protected (FORKID) signature commits to the amount: a prevout without one is an error
    bool threw = false;
    try {
        Call("signrawtransaction " + raw + " " + noAmount + " [" + key1 + "]");
    } catch (const std::runtime_error& e) {
        threw = std::string(e.what()).find("amount") != std::string::npos;
    }
    CHECK(threw);
}

TEST_CASE(rpc_tests, data_outputs) {
    test::TestingSetup setup("regtest");
    const std::string in = "[{\"txid\":\"" + TXID + "\",\"vout\":0}] ";
    CHECK(!Fails("createrawtransaction " + in + "{\"data\":\"00ff00ff\"}"));
    CHECK(!Fails("createrawtransaction " + in + "{\"data\":\"00\",\"data\":\"01\"}")); // several are allowed
    CHECK(Fails("createrawtransaction " + in + "{\"notdata\":\"00ff\"}"));              // not an address either
    CHECK(Fails("createrawtransaction " + in + "{\"data\":\"abc\"}"));                  // odd hex
    CHECK(Fails("createrawtransaction " + in + "{\"data\":\"0g\"}"));
    std::string big;
    for (int i = 0; i < 220; i++) big += strprintf("%02x", i & 0xff);
    const std::string raw = Call("createrawtransaction " + in + "{\"data\":\"" + big + "\"}").get_str();
    UniValue d = Call("decoderawtransaction " + raw);
    const std::string asmStr = find_value(find_value(find_value(d, "vout")[0], "scriptPubKey"), "asm").get_str();
    CHECK(asmStr.compare(0, 9, "OP_RETURN") == 0);
}

TEST_CASE(rpc_tests, monetary_values) {
    // formatting: always eight decimals, sign kept
    CHECK_EQ(ValueFromAmount(0).write(), std::string("0.00000000"));
    CHECK_EQ(ValueFromAmount(-COIN / 10).write(), std::string("-0.10000000"));
    CHECK_EQ(ValueFromAmount(2099999999999999LL).write(), std::string("20999999.99999999"));
    for (int e = 0; e <= 16; e++) {
        int64_t v = 1;
        for (int i = 0; i < e; i++) v *= 10;
        std::string digits = std::to_string(v);
        std::string want = digits.size() > 8 ? digits.substr(0, digits.size() - 8) + "." + digits.substr(digits.size() - 8)
                                             : "0." + std::string(8 - digits.size(), '0') + digits;
        CHECK_EQ(ValueFromAmount(v).write(), want);
        if (v <= MAX_MONEY) CHECK_EQ(AmountFromValue(Num(want)), v); // and back
    }
    // parsing: exact up to 1e-8, any notation, nothing finer, nothing negative, nothing too big
    CHECK_EQ(AmountFromValue(Num("0")), (Amount)0);
    CHECK_EQ(AmountFromValue(Num("0.00000001")), (Amount)1);
    CHECK_EQ(AmountFromValue(Num("1e-8")), (Amount)1);
    CHECK_EQ(AmountFromValue(Num("0.1e-7")), (Amount)1);
    CHECK_EQ(AmountFromValue(Num("0.123456780")), (Amount)12345678);
    CHECK_EQ(AmountFromValue(Num("21000000")), (Amount)2100000000000000LL);
    CHECK_EQ(AmountFromValue(Num("2.1e7")), (Amount)2100000000000000LL);
    for (const char* bad : {"-0.00000001", "0.000000001", "1e-9", "21000000.00000001", "1e+11", "93e+9",
                            "0.00000001000000000001", "-1"}) {
        bool threw = false;
        try {
            AmountFromValue(Num(bad));
        } catch (...) {
            threw = true;
        }
        CHECK(threw);
    }
}

TEST_CASE(rpc_tests, json_parsing) {
    UniValue v;
    CHECK(v.read("[1.0]"));
    CHECK(v.read("{\"a\":[true,false,null,\"s\",-2.5e3]}"));
    CHECK_EQ(v["a"].size(), (size_t)5);
    CHECK(!v.read("[1.0"));
    CHECK(!v.read("[1.0] ]"));
    CHECK(!v.read("[1.0] garbage"));
    CHECK(!v.read("{\"a\":}"));
    CHECK(!v.read("{\"a\" 1}"));
    CHECK(!v.read("[01]"));     // no leading zeros
    CHECK(!v.read("[.5]"));
    CHECK(!v.read("[\"\\x\"]")); // bad escape
    CHECK(v.read(" [ \"caf\\u00e9\" ] "));
    CHECK_EQ(v[0].get_str(), std::string("caf\xc3\xa9"));
}

TEST_CASE(rpc_tests, cli_conversion) {
    // numbers and JSON become typed values where the method expects them, strings stay strings
    UniValue p = RPCConvertValues("generatetoaddress", {"101", "bchreg:qqq"});
    CHECK_EQ(p[0].get_int(), 101);
    CHECK_EQ(p[1].get_str(), std::string("bchreg:qqq"));
    p = RPCConvertValues("generatetoaddress", {"7", "addr", "9000"});
    CHECK_EQ(p[2].get_int(), 9000);
    p = RPCConvertValues("getblock", {"00ff", "false"});
    CHECK(p[1].isFalse());
    p = RPCConvertValues("sendtoaddress", {"addr", "0.5", "comment"});
    CHECK(p[1].isNum());
    CHECK(p[2].isStr());
    p = RPCConvertValues("createrawtransaction", {"[]", "{}"});
    CHECK(p[0].isArray());
    CHECK(p[1].isObject());
    bool threw = false;
    try {
        RPCConvertValues("getblockhash", {"not_json{"});
    } catch (...) {
        threw = true;
    }
    CHECK(threw);
}

} // namespace bcp
