// RPC console command-line parser (see console.h for syntax and parity).
#include "rpc/console.h"

#include "rpc/server.h"

#include <algorithm>
#include <cctype>
#include <stdexcept>
#include <utility>

namespace bcp {

bool IsSensitiveConsoleCommand(const std::string& method) {
    static const char* const kSensitive[] = {"importprivkey", "importmulti", "signmessagewithprivkey",
                                             "signrawtransaction", "walletpassphrase", "walletpassphrasechange",
                                             "encryptwallet"};
    std::string m = method;
    std::transform(m.begin(), m.end(), m.begin(), [](unsigned char c) { return (char)std::tolower(c); });
    for (const char* s : kSensitive)
        if (m == s) return true;
    return false;
}

UniValue ConsoleExecuteRPC(const std::string& method, const std::vector<std::string>& args) {
    JSONRPCRequest req;
    req.strMethod = method;
    req.params = RPCConvertValues(method, args);
    return tableRPC.execute(req);
}

namespace {

[[noreturn]] void Syntax() { throw std::runtime_error("Invalid Syntax"); }

std::string Stringify(const UniValue& v) { return v.isStr() ? v.get_str() : v.write(2); }

// One line, parsed by recursive descent: line := call tail; call := word ( '(' args ')' | args )
// query*; args := (arg (ws | ','))*; arg := word | word '(' ... ')' query* (a nested call).
class LineParser {
public:
    LineParser(const std::string& line, const ConsoleExecutor* exec) : s(line), exec(exec) {}

    std::string Run() {
        SkipSpace();
        if (AtLineEnd()) return "";
        std::string name;
        if (!Word(name)) Syntax();
        const UniValue r = Call(name, pos, /*top=*/true);
        // After the top-level call only stray brackets and blanks may follow ("f()()" is
        // accepted); a second command or any other text is an error.
        while (pos < s.size() && (IsSpace(s[pos]) || s[pos] == '(' || s[pos] == ')' || s[pos] == '\n' || s[pos] == '\r'))
            pos++;
        if (pos < s.size()) Syntax();
        return Stringify(r);
    }

    std::string Filtered() const {
        std::string out = s;
        while (!out.empty() && (out.back() == '\n' || out.back() == '\r')) out.pop_back();
        for (auto it = ranges.rbegin(); it != ranges.rend(); ++it) {
            const size_t b = std::min(it->first, out.size()), e = std::min(it->second, out.size());
            out.replace(b, e - b, "(\xe2\x80\xa6)"); // "(…)"
        }
        return out;
    }

private:
    const std::string& s;
    const ConsoleExecutor* exec;
    size_t pos = 0;
    int sensitiveDepth = 0; // > 0 inside the arguments of a sensitive command
    int callDepth = 0;      // nested calls: bounded so a hostile line cannot exhaust the stack
    static constexpr int MAX_CALL_DEPTH = 64;
    std::vector<std::pair<size_t, size_t>> ranges;

    static bool IsSpace(char c) { return c == ' ' || c == '\t'; }
    bool AtLineEnd() const { return pos >= s.size() || s[pos] == '\n' || s[pos] == '\r'; }
    void SkipSpace() {
        while (pos < s.size() && IsSpace(s[pos])) pos++;
    }

    // A word: bare characters, quoted runs and escapes, up to whitespace, ',', '(', ')' or the
    // end of the line. Returns false if no word starts here.
    bool Word(std::string& out) {
        out.clear();
        bool any = false;
        while (!AtLineEnd()) {
            const char c = s[pos];
            if (IsSpace(c) || c == ',' || c == '(' || c == ')') break;
            any = true;
            pos++;
            if (c == '\'') {
                const size_t close = s.find('\'', pos);
                if (close == std::string::npos) throw std::runtime_error("Parse error: unbalanced ' or \"");
                out.append(s, pos, close - pos);
                pos = close + 1;
            } else if (c == '"') {
                for (;;) {
                    if (pos >= s.size()) throw std::runtime_error("Parse error: unbalanced ' or \"");
                    const char d = s[pos++];
                    if (d == '"') break;
                    if (d == '\\' && pos < s.size()) {
                        const char e = s[pos++];
                        if (e != '"' && e != '\\') out += '\\'; // only \" and \\ are escapes here
                        out += e;
                    } else {
                        out += d;
                    }
                }
            } else if (c == '\\') {
                if (pos >= s.size()) Syntax();
                out += s[pos++];
            } else {
                out += c;
            }
        }
        return any;
    }

    // Arguments up to ')' (consumed) or the end of the line. A comma that directly follows an
    // argument demands another argument before the next comma or the end.
    void Args(std::vector<std::string>& args) {
        bool needArg = false;
        for (;;) {
            SkipSpace();
            if (AtLineEnd()) {
                if (needArg) Syntax();
                return;
            }
            const char c = s[pos];
            if (c == ')') {
                if (needArg) Syntax();
                pos++;
                return;
            }
            if (c == ',') {
                if (needArg) Syntax();
                pos++;
                continue;
            }
            if (c == '(') { // a bracket that does not follow a word opens nothing
                pos++;
                continue;
            }
            std::string w;
            Word(w);
            if (pos < s.size() && s[pos] == '(') {
                const std::string v = Stringify(Call(w, pos, /*top=*/false));
                if (exec && !v.empty()) args.push_back(v);
            } else {
                args.push_back(w);
            }
            needArg = false;
            if (pos < s.size() && s[pos] == ',') {
                pos++;
                needArg = true;
            }
        }
    }

    UniValue Call(const std::string& name, size_t nameEnd, bool top) {
        if (++callDepth > MAX_CALL_DEPTH) Syntax();
        struct DepthGuard {
            int& d;
            ~DepthGuard() { --d; }
        } guard{callDepth};
        const bool opens = sensitiveDepth == 0 && IsSensitiveConsoleCommand(name);
        if (opens || sensitiveDepth > 0) sensitiveDepth++;
        std::vector<std::string> args;
        if (pos < s.size() && s[pos] == '(') {
            pos++;
            Args(args);
        } else if (top) {
            Args(args); // `method arg arg ...` to the end of the line
        }
        UniValue r;
        if (exec) r = (*exec)(name, args);
        Queries(r);
        if (sensitiveDepth > 0) {
            sensitiveDepth--;
            if (opens) ranges.emplace_back(nameEnd, AtLineEnd() && top ? s.size() : pos);
        }
        return r;
    }

    // `[key]` selectors on a call's result: array index or object member.
    void Queries(UniValue& r) {
        while (pos < s.size() && s[pos] == '[') {
            const size_t close = s.find(']', pos + 1);
            if (close == std::string::npos) Syntax();
            const std::string key = s.substr(pos + 1, close - pos - 1);
            pos = close + 1;
            if (!exec || key.empty()) continue;
            UniValue sub;
            if (r.isArray()) {
                for (char ch : key)
                    if (!std::isdigit((unsigned char)ch)) throw std::runtime_error("Invalid result query");
                // an index longer than any array is simply out of range (no stoull overflow)
                const size_t i = key.size() > 18 ? SIZE_MAX : (size_t)std::stoull(key);
                if (i < r.size()) sub = r[i];
            } else if (r.isObject()) {
                sub = find_value(r, key);
            } else {
                throw std::runtime_error("Invalid result query");
            }
            r = sub;
        }
    }
};

} // namespace

void RPCParseCommandLine(std::string& result, const std::string& line, const ConsoleExecutor* exec,
                         std::string* filtered) {
    LineParser p(line, exec);
    result = p.Run();
    if (filtered) *filtered = p.Filtered();
}

} // namespace bcp
