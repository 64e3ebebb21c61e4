#include "util/univalue.h"

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <locale>
#include <sstream>

namespace bcp {

const UniValue UniValue::NullUniValue;

void UniValue::clear() {
    typ = VNULL;
    val.clear();
    keys.clear();
    values.clear();
}
bool UniValue::setNull() {
    clear();
    return true;
}
bool UniValue::setBool(bool v) {
    clear();
    typ = VBOOL;
    if (v) val = "1";
    return true;
}
static bool validNumStr(const std::string& s) {
    // JSON number grammar
    size_t i = 0;
    if (i < s.size() && s[i] == '-') i++;
    if (i >= s.size()) return false;
    if (s[i] == '0') {
        i++;
    } else if (isdigit((unsigned char)s[i])) {
        while (i < s.size() && isdigit((unsigned char)s[i])) i++;
    } else {
        return false;
    }
    if (i < s.size() && s[i] == '.') {
        i++;
        if (i >= s.size() || !isdigit((unsigned char)s[i])) return false;
        while (i < s.size() && isdigit((unsigned char)s[i])) i++;
    }
    if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
        i++;
        if (i < s.size() && (s[i] == '+' || s[i] == '-')) i++;
        if (i >= s.size() || !isdigit((unsigned char)s[i])) return false;
        while (i < s.size() && isdigit((unsigned char)s[i])) i++;
    }
    return i == s.size();
}
bool UniValue::setNumStr(const std::string& v) {
    if (!validNumStr(v)) return false;
    clear();
    typ = VNUM;
    val = v;
    return true;
}
bool UniValue::setInt(uint64_t v) { return setNumStr(std::to_string(v)); }
bool UniValue::setInt(int64_t v) { return setNumStr(std::to_string(v)); }
bool UniValue::setFloat(double v) {
    std::ostringstream oss;
    oss.imbue(std::locale::classic());
    oss.precision(16);
    oss << v;
    return setNumStr(oss.str());
}
bool UniValue::setStr(const std::string& v) {
    clear();
    typ = VSTR;
    val = v;
    return true;
}
bool UniValue::setArray() {
    clear();
    typ = VARR;
    return true;
}
bool UniValue::setObject() {
    clear();
    typ = VOBJ;
    return true;
}
bool UniValue::push_back(const UniValue& v) {
    if (typ != VARR) return false;
    values.push_back(v);
    return true;
}
bool UniValue::push_backV(const std::vector<UniValue>& vec) {
    if (typ != VARR) return false;
    values.insert(values.end(), vec.begin(), vec.end());
    return true;
}
bool UniValue::pushKV(const std::string& key, const UniValue& v) {
    if (typ != VOBJ) return false;
    keys.push_back(key);
    values.push_back(v);
    return true;
}
bool UniValue::pushKVs(const UniValue& obj) {
    if (typ != VOBJ || obj.typ != VOBJ) return false;
    for (size_t i = 0; i < obj.keys.size(); i++) pushKV(obj.keys[i], obj.values[i]);
    return true;
}
const UniValue& UniValue::operator[](const std::string& key) const {
    if (typ != VOBJ) return NullUniValue;
    for (size_t i = 0; i < keys.size(); i++)
        if (keys[i] == key) return values[i];
    return NullUniValue;
}
const UniValue& UniValue::operator[](size_t index) const {
    if (typ != VOBJ && typ != VARR) return NullUniValue;
    if (index >= values.size()) return NullUniValue;
    return values[index];
}
bool UniValue::exists(const std::string& key) const {
    for (const auto& k : keys)
        if (k == key) return true;
    return false;
}
const std::vector<std::string>& UniValue::getKeys() const {
    if (typ != VOBJ) throw std::runtime_error("JSON value is not an object as expected");
    return keys;
}
const std::vector<UniValue>& UniValue::getValues() const {
    if (typ != VOBJ && typ != VARR) throw std::runtime_error("JSON value is not an object or array as expected");
    return values;
}
bool UniValue::get_bool() const {
    if (typ != VBOOL) throw std::runtime_error("JSON value is not a boolean as expected");
    return isTrue();
}
const std::string& UniValue::get_str() const {
    if (typ != VSTR) throw std::runtime_error("JSON value is not a string as expected");
    return val;
}
int UniValue::get_int() const {
    if (typ != VNUM) throw std::runtime_error("JSON value is not an integer as expected");
    errno = 0;
    char* end = nullptr;
    const long long n = strtoll(val.c_str(), &end, 10);
    if (*end != 0 || errno == ERANGE || n < INT32_MIN || n > INT32_MAX) throw std::runtime_error("JSON integer out of range");
    return (int)n;
}
int64_t UniValue::get_int64() const {
    if (typ != VNUM) throw std::runtime_error("JSON value is not an integer as expected");
    errno = 0;
    char* end = nullptr;
    const long long n = strtoll(val.c_str(), &end, 10);
    if (*end != 0 || errno == ERANGE) throw std::runtime_error("JSON integer out of range");
    return (int64_t)n;
}
double UniValue::get_real() const {
    if (typ != VNUM) throw std::runtime_error("JSON value is not a number as expected");
    std::istringstream iss(val);
    iss.imbue(std::locale::classic());
    double d;
    iss >> d;
    if (iss.fail()) throw std::runtime_error("JSON double out of range");
    return d;
}
const UniValue& UniValue::get_obj() const {
    if (typ != VOBJ) throw std::runtime_error("JSON value is not an object as expected");
    return *this;
}
const UniValue& UniValue::get_array() const {
    if (typ != VARR) throw std::runtime_error("JSON value is not an array as expected");
    return *this;
}

std::string JsonEscape(const std::string& s) {
    std::string o;
    o.reserve(s.size() + 2);
    for (unsigned char c : s) {
        switch (c) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\b': o += "\\b"; break;
        case '\f': o += "\\f"; break;
        case '\n': o += "\\n"; break;
        case '\r': o += "\\r"; break;
        case '\t': o += "\\t"; break;
        default:
            if (c < 0x20 || c == 0x7f) {
                char buf[8];
                snprintf(buf, sizeof(buf), "\\u%04x", c);
                o += buf;
            } else {
                o.push_back((char)c);
            }
        }
    }
    return o;
}

static void indentStr(unsigned prettyIndent, unsigned indentLevel, std::string& s) { s.append(prettyIndent * indentLevel, ' '); }

std::string UniValue::write(unsigned prettyIndent, unsigned indentLevel) const {
    std::string s;
    s.reserve(1024);
    const unsigned modIndent = indentLevel ? indentLevel : 1;
    switch (typ) {
    case VNULL: s += "null"; break;
    case VOBJ: writeObject(prettyIndent, modIndent, s); break;
    case VARR: writeArray(prettyIndent, modIndent, s); break;
    case VSTR: s += "\"" + JsonEscape(val) + "\""; break;
    case VNUM: s += val; break;
    case VBOOL: s += (val == "1" ? "true" : "false"); break;
    }
    return s;
}
void UniValue::writeArray(unsigned prettyIndent, unsigned indentLevel, std::string& s) const {
    s += "[";
    if (prettyIndent) s += "\n";
    for (size_t i = 0; i < values.size(); i++) {
        if (prettyIndent) indentStr(prettyIndent, indentLevel, s);
        s += values[i].write(prettyIndent, indentLevel + 1);
        if (i != values.size() - 1) s += ",";
        if (prettyIndent) s += "\n";
    }
    if (prettyIndent) indentStr(prettyIndent, indentLevel - 1, s);
    s += "]";
}
void UniValue::writeObject(unsigned prettyIndent, unsigned indentLevel, std::string& s) const {
    s += "{";
    if (prettyIndent) s += "\n";
    for (size_t i = 0; i < keys.size(); i++) {
        if (prettyIndent) indentStr(prettyIndent, indentLevel, s);
        s += "\"" + JsonEscape(keys[i]) + "\":";
        if (prettyIndent) s += " ";
        s += values[i].write(prettyIndent, indentLevel + 1);
        if (i != values.size() - 1) s += ",";
        if (prettyIndent) s += "\n";
    }
    if (prettyIndent) indentStr(prettyIndent, indentLevel - 1, s);
    s += "}";
}

// ------------------------------------------------------------------ parser
namespace {
struct Parser {
    const char* p;
    const char* end;
    int depth = 0;
    void ws() {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
    }
    static void putUtf8(std::string& o, unsigned cp) {
        if (cp < 0x80) o.push_back((char)cp);
        else if (cp < 0x800) {
            o.push_back((char)(0xC0 | (cp >> 6)));
            o.push_back((char)(0x80 | (cp & 0x3F)));
        } else if (cp < 0x10000) {
            o.push_back((char)(0xE0 | (cp >> 12)));
            o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            o.push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            o.push_back((char)(0xF0 | (cp >> 18)));
            o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            o.push_back((char)(0x80 | (cp & 0x3F)));
        }
    }
    bool hex4(unsigned& out) {
        if (end - p < 4) return false;
        out = 0;
        for (int i = 0; i < 4; i++) {
            const char c = *p++;
            out <<= 4;
            if (c >= '0' && c <= '9') out |= c - '0';
            else if (c >= 'a' && c <= 'f') out |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') out |= c - 'A' + 10;
            else return false;
        }
        return true;
    }
    bool str(std::string& o) {
        if (p >= end || *p != '"') return false;
        p++;
        while (p < end && *p != '"') {
            const unsigned char c = (unsigned char)*p;
            if (c < 0x20) return false;
            if (c == '\\') {
                p++;
                if (p >= end) return false;
                switch (*p++) {
                case '"': o.push_back('"'); break;
                case '\\': o.push_back('\\'); break;
                case '/': o.push_back('/'); break;
                case 'b': o.push_back('\b'); break;
                case 'f': o.push_back('\f'); break;
                case 'n': o.push_back('\n'); break;
                case 'r': o.push_back('\r'); break;
                case 't': o.push_back('\t'); break;
                case 'u': {
                    unsigned cp;
                    if (!hex4(cp)) return false;
                    if (cp >= 0xD800 && cp < 0xDC00) {
                        unsigned lo;
                        if (end - p < 6 || p[0] != '\\' || p[1] != 'u') return false;
                        p += 2;
                        if (!hex4(lo) || lo < 0xDC00 || lo > 0xDFFF) return false;
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    putUtf8(o, cp);
                    break;
                }
                default: return false;
                }
            } else {
                o.push_back((char)c);
                p++;
            }
        }
        if (p >= end) return false;
        p++;
        return true;
    }
    bool value(UniValue& v) {
        ws();
        if (p >= end) return false;
        if (++depth > 512) return false;
        bool ok = false;
        const char c = *p;
        if (c == '{') {
            p++;
            v.setObject();
            ws();
            if (p < end && *p == '}') {
                p++;
                ok = true;
            } else {
                while (true) {
                    ws();
                    std::string k;
                    if (!str(k)) break;
                    ws();
                    if (p >= end || *p != ':') break;
                    p++;
                    UniValue child;
                    if (!value(child)) break;
                    v.pushKV(k, child);
                    ws();
                    if (p < end && *p == ',') {
                        p++;
                        continue;
                    }
                    if (p < end && *p == '}') {
                        p++;
                        ok = true;
                    }
                    break;
                }
            }
        } else if (c == '[') {
            p++;
            v.setArray();
            ws();
            if (p < end && *p == ']') {
                p++;
                ok = true;
            } else {
                while (true) {
                    UniValue child;
                    if (!value(child)) break;
                    v.push_back(child);
                    ws();
                    if (p < end && *p == ',') {
                        p++;
                        continue;
                    }
                    if (p < end && *p == ']') {
                        p++;
                        ok = true;
                    }
                    break;
                }
            }
        } else if (c == '"') {
            std::string s;
            ok = str(s);
            if (ok) v.setStr(s);
        } else if (end - p >= 4 && !strncmp(p, "true", 4)) {
            p += 4;
            v.setBool(true);
            ok = true;
        } else if (end - p >= 5 && !strncmp(p, "false", 5)) {
            p += 5;
            v.setBool(false);
            ok = true;
        } else if (end - p >= 4 && !strncmp(p, "null", 4)) {
            p += 4;
            v.setNull();
            ok = true;
        } else if (c == '-' || (c >= '0' && c <= '9')) {
            const char* s = p;
            while (p < end && (isdigit((unsigned char)*p) || *p == '-' || *p == '+' || *p == '.' || *p == 'e' || *p == 'E'))
                p++;
            ok = v.setNumStr(std::string(s, p));
        }
        depth--;
        return ok;
    }
};
} // namespace

bool UniValue::read(const std::string& raw) {
    clear();
    Parser ps{raw.data(), raw.data() + raw.size()};
    UniValue v;
    if (!ps.value(v)) return false;
    ps.ws();
    if (ps.p != ps.end) return false;
    *this = v;
    return true;
}

const UniValue& find_value(const UniValue& obj, const std::string& name) { return obj[name]; }

const char* uvTypeName(UniValue::VType t) {
    switch (t) {
    case UniValue::VNULL: return "null";
    case UniValue::VBOOL: return "bool";
    case UniValue::VOBJ: return "object";
    case UniValue::VARR: return "array";
    case UniValue::VSTR: return "string";
    case UniValue::VNUM: return "number";
    }
    return nullptr;
}

} // namespace bcp
