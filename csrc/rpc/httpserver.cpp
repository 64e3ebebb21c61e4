#include "rpc/httpserver.h"
#include "crypto/hashes.h"
#include "rpc/server.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <arpa/inet.h>
#include <cerrno>
#include <cstring>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

namespace bcp {

static const char* StatusText(int s) {
    switch (s) {
    case 200: return "OK";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    }
    return "Unknown";
}

HTTPServer::HTTPServer(const Options& o) : opts(o) {}
HTTPServer::~HTTPServer() { Stop(); }

bool HTTPServer::Start(std::string& err) {
    for (const auto& b : opts.bind) {
        struct addrinfo hints, *res = nullptr;
        memset(&hints, 0, sizeof(hints));
        hints.ai_family = AF_UNSPEC;
        hints.ai_socktype = SOCK_STREAM;
        hints.ai_flags = AI_PASSIVE | AI_NUMERICHOST;
        if (getaddrinfo(b.first.c_str(), std::to_string(b.second).c_str(), &hints, &res) != 0 || !res) {
            err = "cannot resolve rpc bind address " + b.first;
            continue;
        }
        const int fd = socket(res->ai_family, SOCK_STREAM, 0);
        int one = 1;
        setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        if (res->ai_family == AF_INET6) setsockopt(fd, IPPROTO_IPV6, IPV6_V6ONLY, &one, sizeof(one));
        if (fd < 0 || bind(fd, res->ai_addr, res->ai_addrlen) != 0 || listen(fd, 64) != 0) {
            err = strprintf("Unable to bind RPC on %s:%d: %s", b.first.c_str(), b.second, strerror(errno));
            if (fd >= 0) close(fd);
            freeaddrinfo(res);
            continue;
        }
        if (boundPort == 0) {
            struct sockaddr_storage ss;
            socklen_t len = sizeof(ss);
            if (getsockname(fd, (struct sockaddr*)&ss, &len) == 0)
                boundPort = ss.ss_family == AF_INET ? ntohs(((struct sockaddr_in*)&ss)->sin_port)
                                                    : ntohs(((struct sockaddr_in6*)&ss)->sin6_port);
        }
        freeaddrinfo(res);
        listenFds.push_back(fd);
    }
    if (listenFds.empty()) return false;
    for (int fd : listenFds) acceptThreads.emplace_back([this, fd] { AcceptLoop(fd); });
    return true;
}

void HTTPServer::Stop() {
    if (stopping.exchange(true)) return;
    for (int fd : listenFds) shutdown(fd, SHUT_RDWR);
    for (auto& t : acceptThreads)
        if (t.joinable()) t.join();
    for (int fd : listenFds) close(fd);
    listenFds.clear();
    {
        std::lock_guard<std::mutex> l(csConns);
        for (int fd : connFds) shutdown(fd, SHUT_RDWR);
    }
    // connection threads are detached: wait for them to drain
    for (int i = 0; i < 1000 && activeConns.load() > 0; i++) MilliSleep(10);
}

void HTTPServer::RegisterHandler(const std::string& prefix, bool exact, HTTPHandler h) {
    std::lock_guard<std::mutex> l(csHandlers);
    handlers.emplace_back(prefix, exact, std::move(h));
}
void HTTPServer::UnregisterHandler(const std::string& prefix) {
    std::lock_guard<std::mutex> l(csHandlers);
    handlers.erase(std::remove_if(handlers.begin(), handlers.end(),
                                  [&](const std::tuple<std::string, bool, HTTPHandler>& t) { return std::get<0>(t) == prefix; }),
                   handlers.end());
}

static bool MatchSubnet(const std::string& peer, const std::string& subnet) {
    std::string net = subnet;
    int bits = -1;
    const size_t slash = net.find('/');
    if (slash != std::string::npos) {
        bits = atoi(net.substr(slash + 1).c_str());
        net = net.substr(0, slash);
    }
    unsigned char a[16], b[16];
    const bool v4 = inet_pton(AF_INET, peer.c_str(), a) == 1;
    if (v4 != (inet_pton(AF_INET, net.c_str(), b) == 1)) {
        if (v4 || inet_pton(AF_INET6, peer.c_str(), a) != 1 || inet_pton(AF_INET6, net.c_str(), b) != 1) return false;
    } else if (!v4 && (inet_pton(AF_INET6, peer.c_str(), a) != 1 || inet_pton(AF_INET6, net.c_str(), b) != 1)) {
        return false;
    }
    const int total = v4 ? 32 : 128;
    if (bits < 0) bits = total;
    for (int i = 0; i < bits; i++) {
        const int byte = i / 8, bit = 7 - (i % 8);
        if (((a[byte] >> bit) & 1) != ((b[byte] >> bit) & 1)) return false;
    }
    return true;
}

bool HTTPServer::Allowed(const std::string& peer) const {
    if (opts.allowSubnets.empty()) return peer == "127.0.0.1" || peer == "::1";
    for (const auto& s : opts.allowSubnets)
        if (MatchSubnet(peer, s)) return true;
    return false;
}

void HTTPServer::AcceptLoop(int lfd) {
    RenameThread("bcp-httpaccept");
    while (!stopping.load()) {
        struct pollfd p = {lfd, POLLIN, 0};
        if (poll(&p, 1, 200) <= 0) continue;
        struct sockaddr_storage ss;
        socklen_t len = sizeof(ss);
        const int fd = accept(lfd, (struct sockaddr*)&ss, &len);
        if (fd < 0) continue;
        char host[INET6_ADDRSTRLEN] = {0};
        if (ss.ss_family == AF_INET) inet_ntop(AF_INET, &((struct sockaddr_in*)&ss)->sin_addr, host, sizeof(host));
        else inet_ntop(AF_INET6, &((struct sockaddr_in6*)&ss)->sin6_addr, host, sizeof(host));
        std::string peer(host);
        if (peer.compare(0, 7, "::ffff:") == 0) peer = peer.substr(7);
        if (!Allowed(peer) || activeConns.load() >= opts.maxConnections) {
            const std::string r = "HTTP/1.1 403 Forbidden\r\nContent-Length: 0\r\nConnection: close\r\n\r\n";
            (void)!write(fd, r.data(), r.size());
            close(fd);
            continue;
        }
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        std::lock_guard<std::mutex> l(csConns);
        activeConns++;
        connFds.push_back(fd);
        std::thread([this, fd, peer] { ServeConnection(fd, peer); }).detach();
    }
}

static bool ReadSome(int fd, std::string& buf, int timeoutMs) {
    struct pollfd p = {fd, POLLIN, 0};
    if (poll(&p, 1, timeoutMs) <= 0) return false;
    char tmp[16384];
    const ssize_t n = read(fd, tmp, sizeof(tmp));
    if (n <= 0) return false;
    buf.append(tmp, (size_t)n);
    return true;
}

static bool WriteAllFd(int fd, const std::string& s) {
    size_t off = 0;
    while (off < s.size()) {
        const ssize_t n = write(fd, s.data() + off, s.size() - off);
        if (n <= 0) {
            if (n < 0 && errno == EINTR) continue;
            return false;
        }
        off += (size_t)n;
    }
    return true;
}

bool HTTPServer::Dispatch(const HTTPRequest& req, HTTPReply& rep) {
    std::string path = req.uri;
    HTTPHandler h;
    {
        std::lock_guard<std::mutex> l(csHandlers);
        for (const auto& t : handlers) {
            const std::string& prefix = std::get<0>(t);
            const bool match = std::get<1>(t) ? path == prefix : path.compare(0, prefix.size(), prefix) == 0;
            if (match) {
                h = std::get<2>(t);
                break;
            }
        }
    }
    if (!h) {
        rep.status = 404;
        rep.body.clear();
        return true;
    }
    return h(req, rep);
}

void HTTPServer::ServeConnection(int fd, std::string peer) {
    RenameThread("bcp-httpworker");
    std::string buf;
    bool keepAlive = true;
    while (keepAlive && !stopping.load()) {
        // headers
        size_t hdrEnd;
        while ((hdrEnd = buf.find("\r\n\r\n")) == std::string::npos) {
            if (buf.size() > 1 << 20 || !ReadSome(fd, buf, opts.timeoutSeconds * 1000)) {
                keepAlive = false;
                break;
            }
        }
        if (!keepAlive) break;
        HTTPRequest req;
        req.peer = peer;
        {
            const std::string head = buf.substr(0, hdrEnd);
            size_t lineEnd = head.find("\r\n");
            const std::string requestLine = head.substr(0, lineEnd);
            std::vector<std::string> parts = SplitString(requestLine, ' ');
            if (parts.size() < 3) break;
            req.method = parts[0];
            req.uri = parts[1];
            req.version = parts[2];
            size_t pos = lineEnd == std::string::npos ? head.size() : lineEnd + 2;
            while (pos < head.size()) {
                size_t e = head.find("\r\n", pos);
                if (e == std::string::npos) e = head.size();
                const std::string line = head.substr(pos, e - pos);
                const size_t colon = line.find(':');
                if (colon != std::string::npos)
                    req.headers[ToLower(TrimString(line.substr(0, colon)))] = TrimString(line.substr(colon + 1));
                pos = e + 2;
            }
        }
        buf.erase(0, hdrEnd + 4);
        const int64_t contentLength = atoi64(req.Header("content-length"));
        if (contentLength < 0 || contentLength > 64 * 1000 * 1000) break;
        while ((int64_t)buf.size() < contentLength)
            if (!ReadSome(fd, buf, opts.timeoutSeconds * 1000)) {
                keepAlive = false;
                break;
            }
        if (!keepAlive) break;
        req.body = buf.substr(0, (size_t)contentLength);
        buf.erase(0, (size_t)contentLength);
        const std::string conn = ToLower(req.Header("connection"));
        keepAlive = req.version == "HTTP/1.1" ? conn != "close" : conn == "keep-alive";
        HTTPReply rep;
        // work queue (reference httpserver.cpp:268-280): -rpcthreads requests run, up to
        // -rpcworkqueue more may wait; anything beyond is answered 500 at once
        if (inFlight.fetch_add(1) >= opts.threads + std::max(opts.workQueueDepth, 1)) {
            LogPrintf("WARNING: request rejected because http work queue depth exceeded, it can be increased with "
                      "the -rpcworkqueue= setting\n");
            rep.status = 500;
            rep.contentType = "text/plain";
            rep.body = "Work queue depth exceeded";
        } else {
            try {
                Dispatch(req, rep);
            } catch (const std::exception& e) {
                rep.status = 500;
                rep.contentType = "text/plain";
                rep.body = e.what();
            }
        }
        inFlight.fetch_sub(1);
        std::string out = strprintf("HTTP/1.1 %d %s\r\n", rep.status, StatusText(rep.status));
        out += "Content-Type: " + rep.contentType + "\r\n";
        out += strprintf("Content-Length: %zu\r\n", rep.body.size());
        for (const auto& h : rep.extraHeaders) out += h.first + ": " + h.second + "\r\n";
        out += keepAlive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n";
        out += rep.body;
        if (!WriteAllFd(fd, out)) break;
    }
    close(fd);
    std::lock_guard<std::mutex> l(csConns);
    connFds.erase(std::remove(connFds.begin(), connFds.end(), fd), connFds.end());
    activeConns--;
}

// ------------------------------------------------------------------ JSON-RPC over HTTP
static std::string strRPCUserColonPass;
static std::vector<std::string> vRPCAuth; // user:salt$hmac

static bool TimingResistantEqual(const std::string& a, const std::string& b) {
    if (b.size() == 0) return a.size() == 0;
    size_t accumulator = a.size() ^ b.size();
    for (size_t i = 0; i < a.size(); i++) accumulator |= a[i] ^ b[i % b.size()];
    return accumulator == 0;
}

static bool CheckUserAuthorized(const std::string& userpass, std::string& user) {
    user = userpass.substr(0, userpass.find(':'));
    if (TimingResistantEqual(userpass, strRPCUserColonPass)) return true;
    const std::string pass = userpass.find(':') == std::string::npos ? "" : userpass.substr(userpass.find(':') + 1);
    for (const std::string& entry : vRPCAuth) {
        // rpcauth=<USERNAME>:<SALT>$<HASH>, HASH = HMAC-SHA256(key=SALT, msg=PASSWORD)
        std::vector<std::string> fields = SplitString(entry, ':');
        if (fields.size() != 2) continue;
        std::vector<std::string> salthash = SplitString(fields[1], '$');
        if (salthash.size() != 2 || fields[0] != user) continue;
        unsigned char out[32];
        CHMAC_SHA256((const unsigned char*)salthash[0].data(), salthash[0].size())
            .Write((const unsigned char*)pass.data(), pass.size())
            .Finalize(out);
        if (TimingResistantEqual(HexStr(out, out + 32), salthash[1])) return true;
    }
    return false;
}

// "Basic <base64 user:pass>" checked against the RPC credentials (also used by the web GUI).
bool RPCAuthorizedHeader(const std::string& auth, std::string& user) {
    if (auth.compare(0, 6, "Basic ") != 0) return false;
    bool invalid = false;
    std::vector<unsigned char> dec = DecodeBase64(TrimString(auth.substr(6)), &invalid);
    return !invalid && CheckUserAuthorized(std::string(dec.begin(), dec.end()), user);
}

// Cross-site request guard. Command-line and library clients never send an Origin header;
// browsers always do on a POST. A browser request is served only if it comes from the page this
// server itself serves (Origin == http://<Host>), is declared JSON, and carries the custom
// X-Requested-With header that a cross-site "simple" request (form/text-plain POST) cannot set.
// This keeps another site open in the same browser from riding on Basic credentials the browser
// cached for the web GUI (which the reference's native Qt wallet never puts in a browser).
bool BrowserRequestAllowed(const HTTPRequest& req, std::string& why) {
    const std::string origin = req.Header("origin");
    if (origin.empty()) return true;
    const std::string host = req.Header("host");
    if (host.empty() || (origin != "http://" + host && origin != "https://" + host)) {
        why = "cross-origin request refused";
        return false;
    }
    const std::string ct = ToLower(req.Header("content-type"));
    if (ct.compare(0, 16, "application/json") != 0) {
        why = "browser requests must be application/json";
        return false;
    }
    if (req.Header("x-requested-with").empty()) {
        why = "browser requests must carry X-Requested-With";
        return false;
    }
    return true;
}

static bool HTTPReq_JSONRPC(const HTTPRequest& req, HTTPReply& rep) {
    if (req.method != "POST") {
        rep.status = 405;
        rep.body = "JSONRPC server handles only POST requests";
        rep.contentType = "text/plain";
        return false;
    }
    std::string why;
    if (!BrowserRequestAllowed(req, why)) {
        LogPrintf("ThreadRPCServer refused browser request from %s: %s\n", req.peer.c_str(), why.c_str());
        rep.status = 403;
        rep.body = why;
        rep.contentType = "text/plain";
        return false;
    }
    const std::string auth = req.Header("authorization");
    if (auth.compare(0, 6, "Basic ") != 0) {
        rep.status = 401;
        rep.extraHeaders["WWW-Authenticate"] = "Basic realm=\"jsonrpc\"";
        rep.body.clear();
        return false;
    }
    std::string user;
    if (!RPCAuthorizedHeader(auth, user)) {
        LogPrintf("ThreadRPCServer incorrect password attempt from %s\n", req.peer.c_str());
        MilliSleep(250); // deter brute-forcing
        rep.status = 401;
        rep.extraHeaders["WWW-Authenticate"] = "Basic realm=\"jsonrpc\"";
        return false;
    }
    int status = 200;
    rep.body = JSONRPCExecute(req.body, user, status);
    rep.status = status;
    rep.contentType = "application/json";
    return true;
}

bool StartHTTPRPC(HTTPServer& server, const std::string& datadir, std::string& err) {
    vRPCAuth = gArgs.GetArgs("-rpcauth");
    if (gArgs.GetArg("-rpcpassword", "") == "") {
        if (!GenerateAuthCookie(datadir, &strRPCUserColonPass)) {
            err = "Unable to create RPC authentication cookie";
            return false;
        }
    } else {
        strRPCUserColonPass = gArgs.GetArg("-rpcuser", "") + ":" + gArgs.GetArg("-rpcpassword", "");
    }
    server.RegisterHandler("/", true, HTTPReq_JSONRPC);
    server.RegisterHandler("/wallet/", false, HTTPReq_JSONRPC);
    return true;
}

void StopHTTPRPC(const std::string& datadir) {
    if (gArgs.GetArg("-rpcpassword", "") == "") DeleteAuthCookie(datadir);
}

// ------------------------------------------------------------------ client
bool HTTPPost(const std::string& host, int port, const std::string& path, const std::string& auth,
              const std::string& body, int& status, std::string& response, int timeoutSeconds) {
    struct addrinfo hints, *res = nullptr;
    memset(&hints, 0, sizeof(hints));
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) return false;
    int fd = -1;
    for (struct addrinfo* ai = res; ai; ai = ai->ai_next) {
        fd = socket(ai->ai_family, SOCK_STREAM, 0);
        if (fd >= 0 && connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) break;
        if (fd >= 0) close(fd);
        fd = -1;
    }
    freeaddrinfo(res);
    if (fd < 0) return false;
    std::string req = "POST " + path + " HTTP/1.1\r\nHost: " + host + "\r\nConnection: close\r\n";
    if (!auth.empty()) req += "Authorization: Basic " + EncodeBase64(auth) + "\r\n";
    req += strprintf("Content-Type: application/json\r\nContent-Length: %zu\r\n\r\n", body.size()) + body;
    if (!WriteAllFd(fd, req)) {
        close(fd);
        return false;
    }
    std::string buf;
    while (ReadSome(fd, buf, timeoutSeconds * 1000)) {
    }
    close(fd);
    const size_t he = buf.find("\r\n\r\n");
    if (he == std::string::npos) return false;
    const std::string head = buf.substr(0, he);
    std::vector<std::string> parts = SplitString(head.substr(0, head.find("\r\n")), ' ');
    if (parts.size() < 2) return false;
    status = atoi(parts[1].c_str());
    response = buf.substr(he + 4);
    return true;
}

} // namespace bcp
