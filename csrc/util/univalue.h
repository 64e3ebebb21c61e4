// JSON value type with parser and writer (RPC/REST payloads).
// Behaviour parity with the reference's vendored UniValue (src/univalue/include/univalue.h):
// numbers are kept as their literal text (exact amounts), object key order is preserved,
// duplicate keys keep the first occurrence on lookup, write(indent) pretty-printing.
#pragma once
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace bcp {

class UniValue {
public:
    enum VType { VNULL, VOBJ, VARR, VSTR, VNUM, VBOOL };

    UniValue() : typ(VNULL) {}
    UniValue(VType t, const std::string& v = std::string()) : typ(t), val(v) {}
    UniValue(uint64_t v) { setInt(v); }
    UniValue(int64_t v) { setInt(v); }
    UniValue(int v) { setInt((int64_t)v); }
    UniValue(unsigned v) { setInt((uint64_t)v); }
    UniValue(bool v) { setBool(v); }
    UniValue(double v) { setFloat(v); }
    UniValue(const std::string& v) { setStr(v); }
    UniValue(const char* v) { setStr(v); }

    void clear();
    bool setNull();
    bool setBool(bool v);
    bool setNumStr(const std::string& v);
    bool setInt(uint64_t v);
    bool setInt(int64_t v);
    bool setFloat(double v);
    bool setStr(const std::string& v);
    bool setArray();
    bool setObject();

    VType getType() const { return typ; }
    const std::string& getValStr() const { return val; }
    bool empty() const { return values.empty(); }
    size_t size() const { return values.size(); }

    bool isNull() const { return typ == VNULL; }
    bool isTrue() const { return typ == VBOOL && val == "1"; }
    bool isFalse() const { return typ == VBOOL && val != "1"; }
    bool isBool() const { return typ == VBOOL; }
    bool isStr() const { return typ == VSTR; }
    bool isNum() const { return typ == VNUM; }
    bool isArray() const { return typ == VARR; }
    bool isObject() const { return typ == VOBJ; }
    bool getBool() const { return isTrue(); }
    // every named key exists with the given type
    bool checkObject(const std::map<std::string, VType>& memberTypes) const {
        for (const auto& m : memberTypes) {
            if (!exists(m.first) || (*this)[m.first].getType() != m.second) return false;
        }
        return true;
    }

    bool push_back(const UniValue& v);
    bool push_backV(const std::vector<UniValue>& vec);
    bool pushKV(const std::string& key, const UniValue& v); // appends (no dedup)
    void __pushKV(const std::string& key, const UniValue& v) { pushKV(key, v); }
    bool pushKVs(const UniValue& obj);

    const UniValue& operator[](const std::string& key) const;
    const UniValue& operator[](size_t index) const;
    bool exists(const std::string& key) const;
    const std::vector<std::string>& getKeys() const;
    const std::vector<UniValue>& getValues() const;

    bool get_bool() const;
    const std::string& get_str() const;
    int get_int() const;
    int64_t get_int64() const;
    double get_real() const;
    const UniValue& get_obj() const;
    const UniValue& get_array() const;

    std::string write(unsigned prettyIndent = 0, unsigned indentLevel = 0) const;
    bool read(const std::string& raw);

    static const UniValue NullUniValue;

private:
    void writeArray(unsigned prettyIndent, unsigned indentLevel, std::string& s) const;
    void writeObject(unsigned prettyIndent, unsigned indentLevel, std::string& s) const;
    VType typ;
    std::string val;
    std::vector<std::string> keys;
    std::vector<UniValue> values;
};

const UniValue& find_value(const UniValue& obj, const std::string& name);
const char* uvTypeName(UniValue::VType t);
std::string JsonEscape(const std::string& s);

} // namespace bcp
