// Tor hidden-service registration through the Tor control port.
// Parity: reference src/torcontrol.cpp: TorControlConnection (line protocol with
// "250-"/"250 " continuation, async replies), TorController (PROTOCOLINFO ->
// AUTHENTICATE via NULL / HASHEDPASSWORD (-torpassword) / COOKIE / SAFECOOKIE
// (AUTHCHALLENGE + HMAC-SHA256 with the two fixed keys) -> ADD_ONION with a persisted
// private key (<datadir>/onion_private_key) -> AddLocal(<id>.onion:port)), reconnect
// with exponential back-off, -listenonion / -torcontrol / -torpassword.
//
// Design: one blocking-socket thread per controller (no libevent).
#include "crypto/hashes.h"
#include "keys/key.h"
#include "net/net.h"
#include "node/node.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <fcntl.h>
#include <poll.h>
#include <unistd.h>

#include <fstream>
#include <mutex>
#include <sstream>

namespace bcp {

static const std::string SAFE_SERVERKEY = "Tor safe cookie authentication server-to-controller hash";
static const std::string SAFE_CLIENTKEY = "Tor safe cookie authentication controller-to-server hash";

struct TorReply {
    int code = 0;
    std::vector<std::string> lines;
};

// Split "KEY=VALUE KEY2=\"quoted value\"" into a map (reference ParseTorReplyMapping).
static std::map<std::string, std::string> ParseMapping(const std::string& s) {
    std::map<std::string, std::string> m;
    size_t i = 0;
    while (i < s.size()) {
        while (i < s.size() && s[i] == ' ') i++;
        const size_t eq = s.find('=', i);
        if (eq == std::string::npos) break;
        const std::string key = s.substr(i, eq - i);
        i = eq + 1;
        std::string value;
        if (i < s.size() && s[i] == '"') {
            i++;
            while (i < s.size() && s[i] != '"') {
                if (s[i] == '\\' && i + 1 < s.size()) i++;
                value += s[i++];
            }
            i++;
        } else {
            while (i < s.size() && s[i] != ' ') value += s[i++];
        }
        m[key] = value;
    }
    return m;
}

class TorController {
public:
    TorController(const std::string& target, const std::string& datadir, int localPort)
        : target(target), datadir(datadir), localPort(localPort) {}
    ~TorController() { Stop(); }
    void Start() {
        th = std::thread([this] {
            RenameThread("bcp-torcontrol");
            Run();
        });
    }
    void Stop() {
        stop = true;
        {
            // fdMu: the control thread may be closing the socket right now (TSan-found race)
            std::lock_guard<std::mutex> l(fdMu);
            if (fd >= 0) shutdown(fd, SHUT_RDWR);
        }
        if (th.joinable()) th.join();
    }

private:
    void CloseFd() {
        std::lock_guard<std::mutex> l(fdMu);
        if (fd >= 0) close(fd);
        fd = -1;
    }
    bool Connect() {
        CService svc;
        if (!Lookup(target, svc, 9051, true)) return false;
        struct sockaddr_storage ss;
        socklen_t len = sizeof(ss);
        svc.GetSockAddr((struct sockaddr*)&ss, &len);
        const int s = socket(((struct sockaddr*)&ss)->sa_family, SOCK_STREAM, IPPROTO_TCP);
        if (s < 0) return false;
        {
            std::lock_guard<std::mutex> l(fdMu);
            fd = s;
        }
        if (stop || connect(s, (struct sockaddr*)&ss, len) != 0) {
            CloseFd();
            return false;
        }
        return true;
    }
    bool Command(const std::string& cmd, TorReply& reply) {
        const std::string line = cmd + "\r\n";
        if (send(fd, line.data(), line.size(), MSG_NOSIGNAL) != (ssize_t)line.size()) return false;
        reply = TorReply();
        for (;;) {
            std::string l;
            if (!ReadLine(l)) return false;
            if (l.size() < 4) return false;
            reply.code = atoi(l.substr(0, 3).c_str());
            reply.lines.push_back(l.substr(4));
            if (l[3] == ' ') return true; // final line; '-' and '+' continue
        }
    }
    bool ReadLine(std::string& out) {
        for (;;) {
            const size_t nl = buf.find("\r\n");
            if (nl != std::string::npos) {
                out = buf.substr(0, nl);
                buf.erase(0, nl + 2);
                return true;
            }
            struct pollfd p = {fd, POLLIN, 0};
            if (poll(&p, 1, 1000) <= 0) {
                if (stop) return false;
                continue;
            }
            char tmp[4096];
            const ssize_t n = recv(fd, tmp, sizeof(tmp), 0);
            if (n <= 0) return false;
            buf.append(tmp, (size_t)n);
        }
    }
    bool Authenticate() {
        TorReply r;
        if (!Command("PROTOCOLINFO 1", r) || r.code != 250) return false;
        std::set<std::string> methods;
        std::string cookiefile;
        for (const std::string& l : r.lines) {
            if (l.compare(0, 5, "AUTH ") == 0) {
                const auto m = ParseMapping(l.substr(5));
                for (const std::string& meth : SplitString(m.count("METHODS") ? m.at("METHODS") : "", ',')) methods.insert(meth);
                if (m.count("COOKIEFILE")) cookiefile = m.at("COOKIEFILE");
            }
        }
        const std::string password = gArgs.GetArg("-torpassword", "");
        if (!password.empty()) {
            if (!methods.count("HASHEDPASSWORD")) return false;
            std::string esc;
            for (char c : password) {
                if (c == '"' || c == '\\') esc += '\\';
                esc += c;
            }
            return Command("AUTHENTICATE \"" + esc + "\"", r) && r.code == 250;
        }
        if (methods.count("NULL")) return Command("AUTHENTICATE", r) && r.code == 250;
        if (methods.count("SAFECOOKIE") || methods.count("COOKIE")) {
            std::ifstream f(cookiefile, std::ios::binary);
            std::string cookie((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
            if (cookie.size() != 32) return false;
            if (!methods.count("SAFECOOKIE"))
                return Command("AUTHENTICATE " + HexStr(cookie), r) && r.code == 250;
            unsigned char clientNonce[32];
            GetRandBytes(clientNonce, 32);
            if (!Command("AUTHCHALLENGE SAFECOOKIE " + HexStr(clientNonce, clientNonce + 32), r) || r.code != 250)
                return false;
            const std::string l = r.lines.empty() ? "" : r.lines[0];
            const size_t sp = l.find(' ');
            const auto m = ParseMapping(sp == std::string::npos ? "" : l.substr(sp + 1));
            if (!m.count("SERVERHASH") || !m.count("SERVERNONCE")) return false;
            const std::vector<unsigned char> serverHash = ParseHex(m.at("SERVERHASH"));
            const std::vector<unsigned char> serverNonce = ParseHex(m.at("SERVERNONCE"));
            auto hmac = [&](const std::string& key) {
                std::vector<unsigned char> msg(cookie.begin(), cookie.end());
                msg.insert(msg.end(), clientNonce, clientNonce + 32);
                msg.insert(msg.end(), serverNonce.begin(), serverNonce.end());
                std::vector<unsigned char> out(32);
                CHMAC_SHA256((const unsigned char*)key.data(), key.size()).Write(msg.data(), msg.size()).Finalize(out.data());
                return out;
            };
            if (hmac(SAFE_SERVERKEY) != serverHash) {
                LogPrintf("tor: ClientNonce/ServerHash mismatch: server is not the real Tor controller\n");
                return false;
            }
            return Command("AUTHENTICATE " + HexStr(hmac(SAFE_CLIENTKEY)), r) && r.code == 250;
        }
        return false;
    }
    bool AddOnion() {
        const std::string keyFile = datadir + "/onion_private_key";
        std::string key = "NEW:RSA1024";
        {
            std::ifstream f(keyFile);
            std::string k;
            if (f && std::getline(f, k) && !k.empty()) key = k;
        }
        const int port = localPort;
        TorReply r;
        if (!Command(strprintf("ADD_ONION %s Port=%d,127.0.0.1:%d", key.c_str(), port, port), r) || r.code != 250)
            return false;
        std::string serviceId, privateKey;
        for (const std::string& l : r.lines) {
            const auto m = ParseMapping(l);
            if (m.count("ServiceID")) serviceId = m.at("ServiceID");
            if (m.count("PrivateKey")) privateKey = m.at("PrivateKey");
        }
        if (serviceId.empty()) return false;
        if (!privateKey.empty()) {
            std::ofstream f(keyFile);
            f << privateKey << "\n";
        }
        CService svc;
        if (Lookup(serviceId + ".onion", svc, port, false)) {
            AddLocal(svc, LOCAL_MANUAL);
            onion = svc;
        }
        LogPrintf("tor: Got service ID %s, advertising service %s\n", serviceId.c_str(), svc.ToString().c_str());
        return true;
    }
    void Run() {
        int64_t backoff = 1000;
        while (!stop) {
            if (Connect()) {
                buf.clear();
                if (Authenticate() && AddOnion()) {
                    backoff = 1000;
                    // stay connected; the onion lives as long as the control connection
                    std::string l;
                    while (!stop && ReadLine(l)) {
                    }
                } else {
                    LogPrintf("tor: authentication or ADD_ONION failed on %s\n", target.c_str());
                }
                if (onion.IsValid()) RemoveLocal(onion);
                CloseFd();
            } else {
                LogPrint(BCLog::TOR, "tor: Error connecting to Tor control socket %s\n", target.c_str());
            }
            for (int64_t t = 0; t < backoff && !stop; t += 100) MilliSleep(100);
            backoff = std::min<int64_t>(backoff * 3 / 2, 600000);
        }
    }

    std::string target, datadir;
    int localPort;
    std::atomic<bool> stop{false};
    std::thread th;
    std::mutex fdMu; // fd is closed by the control thread and shut down by Stop()
    int fd = -1;
    std::string buf;
    CService onion;
};

static std::unique_ptr<TorController> g_tor;

void StartTorControl(NodeContext& node, int listenPort) {
    if (!gArgs.GetBoolArg("-listenonion", true) || !gArgs.GetBoolArg("-listen", true)) return;
    const std::string target = gArgs.GetArg("-torcontrol", "127.0.0.1:9051");
    g_tor.reset(new TorController(target, node.datadir, listenPort));
    g_tor->Start();
}

void StopTorControl() { g_tor.reset(); }

} // namespace bcp
