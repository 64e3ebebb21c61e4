// bcp-seeder: P2P network crawler + authoritative DNS server for seed hostnames.
// Parity: reference src/seeder/ (main.cpp: crawler threads, DNS thread, dumper and
// stats threads; bitcoin.cpp CSeederNode: version/verack/getaddr handshake and addr
// harvesting; db.{h,cpp} CAddrDb: per-address reliability statistics and "good" node
// selection; dns.cpp: A/AAAA/NS/SOA answers for the seed zone).
//
//   bcp-seeder -host=seed.example.org -ns=ns.example.org [-port=53] [-threads=16]
//              [-seed=ip:port ...] [-testnet|-regtest] [-dumpfile=dnsseed.dump] [-allowlocal]
#include "consensus/params.h"
#include "keys/key.h"
#include "net/protocol.h"
#include "primitives/block.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <arpa/inet.h>
#include <poll.h>
#include <unistd.h>

#include <atomic>
#include <csignal>
#include <cstdio>
#include <fstream>
#include <map>
#include <mutex>
#include <random>
#include <set>
#include <thread>
#include <vector>

using namespace bcp;

// ------------------------------------------------------------------ address database
struct AddrStat {
    CAddress addr;
    int64_t lastTry = 0, lastSuccess = 0;
    int total = 0, success = 0;
    double reliability = 0.0; // EWMA of success (2h half-life style)
    int clientVersion = 0, blocks = 0;
    uint64_t services = 0;
    std::string subver;
    bool IsGood(int64_t now, int minHeight) const {
        if (!success) return false;
        if (!(services & NODE_NETWORK)) return false;
        if (blocks < minHeight) return false;
        if (now - lastSuccess > 24 * 3600) return false;
        return reliability > 0.5 || (total <= 2 && success == total);
    }
};

class SeederDb {
public:
    void Add(const CAddress& a) {
        std::lock_guard<std::mutex> l(cs);
        auto it = db.find((CService)a);
        if (it == db.end()) {
            AddrStat s;
            s.addr = a;
            db.emplace((CService)a, s);
            queue.push_back((CService)a);
        }
    }
    bool Next(CService& out, int64_t now) {
        std::lock_guard<std::mutex> l(cs);
        // newly learned first, then re-test the least recently tried
        while (!queue.empty()) {
            out = queue.front();
            queue.erase(queue.begin());
            if (db[out].lastTry == 0) return true;
        }
        const AddrStat* best = nullptr;
        for (const auto& kv : db)
            if (now - kv.second.lastTry > retryInterval && (!best || kv.second.lastTry < best->lastTry)) best = &kv.second;
        if (!best) return false;
        out = best->addr;
        return true;
    }
    void Result(const CService& s, bool ok, int version, int blocks, uint64_t services, const std::string& subver,
                int64_t now) {
        std::lock_guard<std::mutex> l(cs);
        AddrStat& st = db[s];
        st.addr = CAddress(s, services);
        st.lastTry = now;
        st.total++;
        const double w = 0.2;
        st.reliability = st.reliability * (1 - w) + (ok ? w : 0.0);
        if (ok) {
            st.success++;
            st.lastSuccess = now;
            st.clientVersion = version;
            st.blocks = blocks;
            st.services = services;
            st.subver = subver;
        }
    }
    std::vector<CService> Good(int64_t now, int minHeight, bool ipv6) {
        std::lock_guard<std::mutex> l(cs);
        std::vector<CService> r;
        for (const auto& kv : db)
            if (kv.second.IsGood(now, minHeight) && (kv.first.IsIPv4() != ipv6)) r.push_back(kv.first);
        return r;
    }
    void Dump(const std::string& path, int64_t now) {
        std::lock_guard<std::mutex> l(cs);
        FILE* f = fopen((path + ".new").c_str(), "w");
        if (!f) return;
        fprintf(f, "# address                                        good  lastSuccess    %%(2h)  blocks      svcs  version\n");
        for (const auto& kv : db) {
            const AddrStat& s = kv.second;
            fprintf(f, "%-47s  %4d  %11lld  %6.2f%%  %6d  %08llx  %5d \"%s\"\n", kv.first.ToString().c_str(),
                    (int)s.IsGood(now, 0), (long long)s.lastSuccess, 100.0 * s.reliability, s.blocks,
                    (unsigned long long)s.services, s.clientVersion, s.subver.c_str());
        }
        fclose(f);
        rename((path + ".new").c_str(), path.c_str());
    }
    void Stats(int& total, int& good, int64_t now) {
        std::lock_guard<std::mutex> l(cs);
        total = (int)db.size();
        good = 0;
        for (const auto& kv : db) good += kv.second.IsGood(now, 0);
    }
    int64_t retryInterval = 15 * 60;

private:
    std::mutex cs;
    std::map<CService, AddrStat> db;
    std::vector<CService> queue;
};

// ------------------------------------------------------------------ crawler
static bool SendMsg(int fd, const std::string& cmd, const std::vector<unsigned char>& payload) {
    CMessageHeader hdr(Params().NetMagic(), cmd.c_str(), (uint32_t)payload.size());
    MessageChecksum(payload.data(), payload.size(), hdr.checksum.data());
    std::vector<unsigned char> wire;
    VectorWriter w(wire);
    w << hdr;
    wire.insert(wire.end(), payload.begin(), payload.end());
    return send(fd, wire.data(), wire.size(), MSG_NOSIGNAL) == (ssize_t)wire.size();
}

static bool RecvMsg(int fd, std::string& buf, std::string& cmd, std::vector<unsigned char>& payload, int timeoutMs) {
    const int64_t deadline = GetTimeMillis() + timeoutMs;
    for (;;) {
        if (buf.size() >= CMessageHeader::HEADER_SIZE) {
            CMessageHeader hdr;
            SpanReader r((const unsigned char*)buf.data(), CMessageHeader::HEADER_SIZE);
            r >> hdr;
            if (!hdr.IsValid(Params().NetMagic())) return false;
            if (buf.size() >= CMessageHeader::HEADER_SIZE + hdr.nMessageSize) {
                cmd = hdr.GetCommand();
                payload.assign(buf.begin() + CMessageHeader::HEADER_SIZE,
                               buf.begin() + CMessageHeader::HEADER_SIZE + hdr.nMessageSize);
                buf.erase(0, CMessageHeader::HEADER_SIZE + hdr.nMessageSize);
                return true;
            }
        }
        const int64_t left = deadline - GetTimeMillis();
        if (left <= 0) return false;
        struct pollfd p = {fd, POLLIN, 0};
        if (poll(&p, 1, (int)left) <= 0) return false;
        char tmp[65536];
        const ssize_t n = recv(fd, tmp, sizeof(tmp), 0);
        if (n <= 0) return false;
        buf.append(tmp, (size_t)n);
    }
}

// One crawl: handshake, getaddr, harvest addr messages for a few seconds.
static bool Crawl(const CService& target, SeederDb& db, int& version, int& blocks, uint64_t& services,
                  std::string& subver, std::vector<CAddress>& learned) {
    struct sockaddr_storage ss;
    socklen_t len = sizeof(ss);
    if (!target.GetSockAddr((struct sockaddr*)&ss, &len)) return false;
    const int fd = socket(((struct sockaddr*)&ss)->sa_family, SOCK_STREAM, IPPROTO_TCP);
    if (fd < 0) return false;
    struct timeval tv = {5, 0};
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    bool ok = false;
    if (connect(fd, (struct sockaddr*)&ss, len) == 0) {
        std::vector<unsigned char> p;
        {
            VectorWriter w(p, SER_NETWORK, INIT_PROTO_VERSION);
            const CAddress you(target, NODE_NONE), me(CService(), NODE_NONE);
            uint64_t nonce;
            GetRandBytes((unsigned char*)&nonce, 8);
            w << PROTOCOL_VERSION << (uint64_t)NODE_NONE << (int64_t)GetTime() << you << me << nonce
              << std::string("/bcp-seeder:0.1/") << (int32_t)0 << false;
        }
        std::string buf, cmd;
        std::vector<unsigned char> payload;
        if (SendMsg(fd, NetMsgType::VERSION, p)) {
            const int64_t end = GetTimeMillis() + 10000;
            bool sentGetaddr = false;
            while (GetTimeMillis() < end && RecvMsg(fd, buf, cmd, payload, 3000)) {
                SpanReader r(payload.data(), payload.size(), SER_NETWORK, INIT_PROTO_VERSION);
                try {
                    if (cmd == NetMsgType::VERSION) {
                        CAddress a, b;
                        int64_t t;
                        r >> version >> services >> t >> a;
                        if (!r.empty()) {
                            uint64_t nonce;
                            r >> b >> nonce;
                        }
                        if (!r.empty()) {
                            const uint64_t n = ReadCompactSize(r);
                            subver.resize(std::min<uint64_t>(n, 256));
                            if (n) r.read(&subver[0], subver.size());
                        }
                        if (!r.empty()) r >> blocks;
                        SendMsg(fd, NetMsgType::VERACK, {});
                    } else if (cmd == NetMsgType::VERACK) {
                        ok = true;
                        if (!sentGetaddr) {
                            SendMsg(fd, NetMsgType::GETADDR, {});
                            sentGetaddr = true;
                        }
                    } else if (cmd == NetMsgType::PING) {
                        SendMsg(fd, NetMsgType::PONG, payload);
                    } else if (cmd == NetMsgType::ADDR) {
                        SpanReader ra(payload.data(), payload.size(), SER_NETWORK, PROTOCOL_VERSION);
                        std::vector<CAddress> v;
                        ra >> v;
                        learned.insert(learned.end(), v.begin(), v.end());
                        if (v.size() > 1) break; // got the getaddr reply
                    }
                } catch (const std::exception&) {
                    break;
                }
            }
        }
    }
    close(fd);
    return ok;
}

// ------------------------------------------------------------------ DNS
static std::string g_host, g_ns, g_mbox;
static bool g_allowLocal = false;

static bool ReadName(const unsigned char* p, size_t n, size_t& off, std::string& out) {
    out.clear();
    int jumps = 0;
    size_t pos = off;
    bool jumped = false;
    while (pos < n) {
        const unsigned char l = p[pos];
        if (l == 0) {
            if (!jumped) off = pos + 1;
            return true;
        }
        if ((l & 0xC0) == 0xC0) {
            if (pos + 1 >= n || ++jumps > 10) return false;
            if (!jumped) off = pos + 2;
            pos = ((l & 0x3F) << 8) | p[pos + 1];
            jumped = true;
            continue;
        }
        if (pos + 1 + l > n) return false;
        if (!out.empty()) out += '.';
        out.append((const char*)p + pos + 1, l);
        pos += 1 + l;
    }
    return false;
}

static void PutName(std::vector<unsigned char>& o, const std::string& name) {
    size_t start = 0;
    while (start < name.size()) {
        size_t dot = name.find('.', start);
        if (dot == std::string::npos) dot = name.size();
        o.push_back((unsigned char)(dot - start));
        o.insert(o.end(), name.begin() + start, name.begin() + dot);
        start = dot + 1;
    }
    o.push_back(0);
}

static void Put16(std::vector<unsigned char>& o, uint16_t v) {
    o.push_back(v >> 8);
    o.push_back(v & 0xFF);
}
static void Put32(std::vector<unsigned char>& o, uint32_t v) {
    Put16(o, v >> 16);
    Put16(o, v & 0xFFFF);
}

static std::vector<unsigned char> DnsAnswer(const unsigned char* q, size_t n, SeederDb& db, int minHeight) {
    std::vector<unsigned char> r;
    if (n < 12) return r;
    const uint16_t id = (q[0] << 8) | q[1];
    const uint16_t qd = (q[4] << 8) | q[5];
    size_t off = 12;
    std::string name;
    if (qd != 1 || !ReadName(q, n, off, name) || off + 4 > n) return r;
    const uint16_t qtype = (q[off] << 8) | q[off + 1];
    const uint16_t qclass = (q[off + 2] << 8) | q[off + 3];
    const size_t qend = off + 4;
    const bool inZone = ToLower(name) == ToLower(g_host);
    Put16(r, id);
    Put16(r, inZone ? 0x8400 : 0x8405); // response, authoritative; REFUSED when out of zone
    Put16(r, 1);
    const size_t ancountPos = r.size();
    Put16(r, 0);
    Put16(r, 0);
    Put16(r, 0);
    r.insert(r.end(), q + 12, q + qend);
    if (!inZone || qclass != 1) return r;
    uint16_t ancount = 0;
    auto answerHeader = [&](uint16_t type, uint32_t ttl) {
        Put16(r, 0xC00C); // pointer to the question name
        Put16(r, type);
        Put16(r, 1);
        Put32(r, ttl);
    };
    if (qtype == 1 || qtype == 28 || qtype == 255) {
        const int64_t now = GetTime();
        std::vector<CService> good;
        if (qtype != 28) {
            std::vector<CService> g4 = db.Good(now, minHeight, false);
            good.insert(good.end(), g4.begin(), g4.end());
        }
        if (qtype != 1) {
            std::vector<CService> g6 = db.Good(now, minHeight, true);
            good.insert(good.end(), g6.begin(), g6.end());
        }
        std::shuffle(good.begin(), good.end(), std::mt19937((unsigned)GetRand(UINT32_MAX)));
        for (const CService& s : good) {
            if (ancount >= 20) break;
            if (!g_allowLocal && !s.IsRoutable()) continue;
            if (s.IsIPv4()) {
                answerHeader(1, 3600);
                Put16(r, 4);
                const uint32_t a = s.GetIPv4();
                Put32(r, a);
            } else {
                answerHeader(28, 3600);
                Put16(r, 16);
                r.insert(r.end(), s.Raw(), s.Raw() + 16);
            }
            ancount++;
        }
    }
    if ((qtype == 2 || qtype == 255) && !g_ns.empty()) {
        answerHeader(2, 40000);
        std::vector<unsigned char> nm;
        PutName(nm, g_ns);
        Put16(r, (uint16_t)nm.size());
        r.insert(r.end(), nm.begin(), nm.end());
        ancount++;
    }
    if ((qtype == 6 || qtype == 255) && !g_ns.empty()) {
        answerHeader(6, 40000);
        std::vector<unsigned char> rd;
        PutName(rd, g_ns);
        PutName(rd, g_mbox.empty() ? "hostmaster." + g_host : g_mbox);
        Put32(rd, (uint32_t)GetTime());
        Put32(rd, 604800);
        Put32(rd, 86400);
        Put32(rd, 2592000);
        Put32(rd, 604800);
        Put16(r, (uint16_t)rd.size());
        r.insert(r.end(), rd.begin(), rd.end());
        ancount++;
    }
    r[ancountPos] = ancount >> 8;
    r[ancountPos + 1] = ancount & 0xFF;
    return r;
}

static std::atomic<bool> g_stop{false};
static void OnSignal(int) { g_stop = true; }

int main(int argc, char* argv[]) {
    gArgs.ParseParameters(argc, argv);
    if (gArgs.IsArgSet("-?") || gArgs.IsArgSet("-h") || gArgs.IsArgSet("-help") || !gArgs.IsArgSet("-host")) {
        printf("Usage: bcp-seeder -host=<host> -ns=<ns> [-mbox=<mail>] [-port=<dns port>] [-threads=<n>]\n"
               "                  [-seed=<ip:port>]... [-testnet|-regtest] [-dumpfile=<file>] [-allowlocal]\n"
               "                  [-minheight=<n>] [-retry=<seconds>] [-dumpinterval=<seconds>]\n");
        return gArgs.IsArgSet("-host") ? 0 : 1;
    }
    SelectParams(gArgs.GetChainName());
    g_host = gArgs.GetArg("-host", "");
    g_ns = gArgs.GetArg("-ns", "");
    g_mbox = gArgs.GetArg("-mbox", "");
    g_allowLocal = gArgs.GetBoolArg("-allowlocal", false);
    const int nThreads = (int)gArgs.GetArg("-threads", (int64_t)16);
    const int dnsPort = (int)gArgs.GetArg("-port", (int64_t)53);
    const int minHeight = (int)gArgs.GetArg("-minheight", (int64_t)0);
    const std::string dumpfile = gArgs.GetArg("-dumpfile", "dnsseed.dump");
    signal(SIGINT, OnSignal);
    signal(SIGTERM, OnSignal);
    signal(SIGPIPE, SIG_IGN);

    SeederDb db;
    db.retryInterval = gArgs.GetArg("-retry", (int64_t)15 * 60);
    for (const std::string& s : gArgs.GetArgs("-seed")) {
        CService svc;
        if (Lookup(s, svc, Params().GetDefaultPort(), true)) db.Add(CAddress(svc, NODE_NETWORK));
    }
    for (const CDNSSeedData& seed : Params().DNSSeeds()) {
        std::vector<CNetAddr> ips;
        if (LookupHost(seed.host, ips, 64, true))
            for (const CNetAddr& ip : ips) db.Add(CAddress(CService(ip, (uint16_t)Params().GetDefaultPort()), NODE_NETWORK));
    }

    // DNS thread (UDP)
    const int ufd = socket(AF_INET, SOCK_DGRAM, 0);
    struct sockaddr_in sa = {};
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)dnsPort);
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    if (ufd < 0 || bind(ufd, (struct sockaddr*)&sa, sizeof(sa)) != 0) {
        fprintf(stderr, "Error: cannot bind DNS port %d: %s\n", dnsPort, strerror(errno));
        return 1;
    }
    std::thread dns([&] {
        unsigned char buf[1500];
        while (!g_stop) {
            struct pollfd p = {ufd, POLLIN, 0};
            if (poll(&p, 1, 200) <= 0) continue;
            struct sockaddr_storage from;
            socklen_t fl = sizeof(from);
            const ssize_t n = recvfrom(ufd, buf, sizeof(buf), 0, (struct sockaddr*)&from, &fl);
            if (n <= 0) continue;
            const std::vector<unsigned char> ans = DnsAnswer(buf, (size_t)n, db, minHeight);
            if (!ans.empty()) sendto(ufd, ans.data(), ans.size(), 0, (struct sockaddr*)&from, fl);
        }
    });
    // crawler threads
    std::vector<std::thread> crawlers;
    for (int t = 0; t < nThreads; t++)
        crawlers.emplace_back([&] {
            while (!g_stop) {
                CService target;
                if (!db.Next(target, GetTime())) {
                    MilliSleep(500);
                    continue;
                }
                int version = 0, blocks = 0;
                uint64_t services = 0;
                std::string subver;
                std::vector<CAddress> learned;
                const bool ok = Crawl(target, db, version, blocks, services, subver, learned);
                db.Result(target, ok, version, blocks, services, subver, GetTime());
                for (const CAddress& a : learned)
                    if (g_allowLocal || a.IsRoutable()) db.Add(a);
            }
        });
    // dumper + stats (main thread)
    int64_t nextDump = GetTime() + 5;
    while (!g_stop) {
        MilliSleep(200);
        if (GetTime() >= nextDump) {
            db.Dump(dumpfile, GetTime());
            int total, good;
            db.Stats(total, good, GetTime());
            printf("[%lld] %d/%d available\n", (long long)GetTime(), good, total);
            fflush(stdout);
            nextDump = GetTime() + (int64_t)gArgs.GetArg("-dumpinterval", (int64_t)100);
        }
    }
    dns.join();
    for (auto& t : crawlers) t.join();
    db.Dump(dumpfile, GetTime());
    close(ufd);
    return 0;
}
