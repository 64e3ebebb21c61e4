// univalue_tests: constructors from every scalar type, typed getters and their exceptions
// (range of get_int/get_int64, wrong-type access), setters, arrays, objects (pushKV/pushKVs,
// lookup, exists, checkObject) and read/write round trips, including trailing-garbage rejects.
// Parity: reference src/test/univalue_tests.cpp (univalue_constructor, univalue_typecheck,
// univalue_set, univalue_array, univalue_object, univalue_readwrite).
#include "test/unittest.h"

#include "util/univalue.h"

#include <map>

using namespace bcp;

TEST_CASE(univalue_tests, univalue_constructor) {
    UniValue v1;
    CHECK(v1.isNull());
    UniValue v2(UniValue::VSTR);
    CHECK(v2.isStr());
    UniValue v3(UniValue::VSTR, "foo");
    CHECK(v3.isStr());
    CHECK_EQ(v3.getValStr(), std::string("foo"));
    UniValue numTest;
    CHECK(numTest.setNumStr("82"));
    CHECK(numTest.isNum());
    CHECK_EQ(numTest.getValStr(), std::string("82"));
    UniValue v4((uint64_t)82);
    CHECK(v4.isNum() && v4.getValStr() == "82");
    UniValue v5((int64_t)-82);
    CHECK(v5.isNum() && v5.getValStr() == "-82");
    UniValue v6(-688);
    CHECK(v6.isNum() && v6.getValStr() == "-688");
    UniValue v7(-7.21);
    CHECK(v7.isNum());
    CHECK_EQ(v7.getValStr(), std::string("-7.21"));
    UniValue v8(std::string("yawn"));
    CHECK(v8.isStr() && v8.getValStr() == "yawn");
    UniValue v9("zappa");
    CHECK(v9.isStr() && v9.getValStr() == "zappa");
}

TEST_CASE(univalue_tests, univalue_typecheck) {
    UniValue v1;
    CHECK(v1.setNumStr("1"));
    CHECK(v1.isNum());
    CHECK_THROWS(v1.get_bool());
    UniValue v2;
    CHECK(v2.setBool(true));
    CHECK_EQ(v2.get_bool(), true);
    CHECK_THROWS(v2.get_int());
    UniValue v3;
    CHECK(v3.setNumStr("32482348723847471234"));
    CHECK_THROWS(v3.get_int64());
    CHECK(v3.setNumStr("1000"));
    CHECK_EQ(v3.get_int64(), (int64_t)1000);
    UniValue v4;
    CHECK(v4.setNumStr("2147483648"));
    CHECK_EQ(v4.get_int64(), (int64_t)2147483648LL);
    CHECK_THROWS(v4.get_int());
    CHECK(v4.setNumStr("1000"));
    CHECK_EQ(v4.get_int(), 1000);
    CHECK_THROWS(v4.get_str());
    CHECK_EQ(v4.get_real(), 1000.0);
    CHECK_THROWS(v4.get_array());
    CHECK_THROWS(v4.getKeys());
    CHECK_THROWS(v4.getValues());
    CHECK_THROWS(v4.get_obj());
    UniValue v5;
    CHECK(v5.read("[true, 10]"));
    v5.get_array();
    const std::vector<UniValue> vals = v5.getValues();
    CHECK_THROWS(vals[0].get_int());
    CHECK_EQ(vals[0].get_bool(), true);
    CHECK_EQ(vals[1].get_int(), 10);
    CHECK_THROWS(vals[1].get_bool());
}

TEST_CASE(univalue_tests, univalue_set) {
    UniValue v(UniValue::VSTR, "foo");
    v.clear();
    CHECK(v.isNull());
    CHECK_EQ(v.getValStr(), std::string(""));
    CHECK(v.setObject());
    CHECK(v.isObject());
    CHECK_EQ(v.size(), (size_t)0);
    CHECK(v.getType() == UniValue::VOBJ);
    CHECK(v.empty());
    CHECK(v.setArray());
    CHECK(v.isArray());
    CHECK_EQ(v.size(), (size_t)0);
    CHECK(v.setStr("zum"));
    CHECK(v.isStr() && v.getValStr() == "zum");
    CHECK(v.setFloat(-1.01));
    CHECK(v.isNum());
    CHECK_EQ(v.getValStr(), std::string("-1.01"));
    CHECK(v.setInt((int64_t)1023));
    CHECK_EQ(v.getValStr(), std::string("1023"));
    CHECK(v.setInt((int64_t)-1023LL));
    CHECK_EQ(v.getValStr(), std::string("-1023"));
    CHECK(v.setInt((uint64_t)1023ULL));
    CHECK_EQ(v.getValStr(), std::string("1023"));
    CHECK(v.setNumStr("-688"));
    CHECK(v.isNum() && v.getValStr() == "-688");
    CHECK(v.setBool(false));
    CHECK(v.isBool() && !v.isTrue() && v.isFalse() && !v.getBool());
    CHECK(v.setBool(true));
    CHECK(v.isBool() && v.isTrue() && !v.isFalse() && v.getBool());
    CHECK(!v.setNumStr("zombocom"));
    CHECK(v.setNull());
    CHECK(v.isNull());
}

TEST_CASE(univalue_tests, univalue_array) {
    UniValue arr(UniValue::VARR);
    UniValue v((int64_t)1023LL);
    CHECK(arr.push_back(v));
    CHECK(arr.push_back(std::string("zippy")));
    CHECK(arr.push_back("pippy"));
    std::vector<UniValue> vec;
    v.setStr("boing");
    vec.push_back(v);
    v.setStr("going");
    vec.push_back(v);
    CHECK(arr.push_backV(vec));
    CHECK(!arr.empty());
    CHECK_EQ(arr.size(), (size_t)5);
    CHECK_EQ(arr[0].getValStr(), std::string("1023"));
    CHECK_EQ(arr[1].getValStr(), std::string("zippy"));
    CHECK_EQ(arr[2].getValStr(), std::string("pippy"));
    CHECK_EQ(arr[3].getValStr(), std::string("boing"));
    CHECK_EQ(arr[4].getValStr(), std::string("going"));
    CHECK_EQ(arr[999].getValStr(), std::string(""));
    arr.clear();
    CHECK(arr.empty());
    CHECK_EQ(arr.size(), (size_t)0);
}

TEST_CASE(univalue_tests, univalue_object) {
    UniValue obj(UniValue::VOBJ);
    UniValue v;
    v.setInt((int64_t)100);
    CHECK(obj.pushKV("age", v));
    CHECK(obj.pushKV("first", std::string("John")));
    CHECK(obj.pushKV("last", "Smith"));
    CHECK(obj.pushKV("distance", (int64_t)25));
    CHECK(obj.pushKV("time", (uint64_t)3600));
    CHECK(obj.pushKV("calories", 12));
    CHECK(obj.pushKV("temperature", 90.012));
    UniValue obj2(UniValue::VOBJ);
    CHECK(obj2.pushKV("cat1", 9000));
    CHECK(obj2.pushKV("cat2", 12345));
    CHECK(obj.pushKVs(obj2));
    CHECK(!obj.empty());
    CHECK_EQ(obj.size(), (size_t)9);
    const std::map<std::string, std::string> want = {
        {"age", "100"}, {"first", "John"}, {"last", "Smith"}, {"distance", "25"}, {"time", "3600"},
        {"calories", "12"}, {"temperature", "90.012"}, {"cat1", "9000"}, {"cat2", "12345"}};
    for (const auto& kv : want) {
        CHECK_EQ(obj[kv.first].getValStr(), kv.second);
        CHECK(obj.exists(kv.first));
    }
    CHECK_EQ(obj["nyuknyuknyuk"].getValStr(), std::string(""));
    CHECK(!obj.exists("nyuknyuknyuk"));
    std::map<std::string, UniValue::VType> types;
    for (const char* k : {"age", "distance", "time", "calories", "temperature", "cat1", "cat2"}) types[k] = UniValue::VNUM;
    types["first"] = types["last"] = UniValue::VSTR;
    CHECK(obj.checkObject(types));
    types["cat2"] = UniValue::VSTR;
    CHECK(!obj.checkObject(types));
    obj.clear();
    CHECK(obj.empty());
    CHECK_EQ(obj.size(), (size_t)0);
}

TEST_CASE(univalue_tests, univalue_readwrite) {
    static const char* json1 =
        "[1.10000000,{\"key1\":\"str\\u0000\",\"key2\":800,\"key3\":{\"name\":\"martian http://test.com\"}}]";
    UniValue v;
    CHECK(v.read(json1));
    const std::string strJson1(json1);
    CHECK(v.read(strJson1));
    CHECK(v.isArray());
    CHECK_EQ(v.size(), (size_t)2);
    CHECK_EQ(v[0].getValStr(), std::string("1.10000000"));
    const UniValue obj = v[1];
    CHECK(obj.isObject());
    CHECK_EQ(obj.size(), (size_t)3);
    CHECK(obj["key1"].isStr());
    std::string correct("str");
    correct.push_back('\0');
    CHECK(obj["key1"].getValStr() == correct);
    CHECK(obj["key2"].isNum());
    CHECK_EQ(obj["key2"].getValStr(), std::string("800"));
    CHECK(obj["key3"].isObject());
    CHECK_EQ(strJson1, v.write());
    // whitespace around one value is fine; anything else after it is an error
    CHECK(v.read("  {}\n  "));
    CHECK(v.isObject());
    CHECK(v.read("  []\n  "));
    CHECK(v.isArray());
    CHECK(!v.read("@{}"));
    CHECK(!v.read("{} garbage"));
    CHECK(!v.read("[]{}"));
    CHECK(!v.read("{}[]"));
    CHECK(!v.read("{} 42"));
}
