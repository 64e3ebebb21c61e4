// HTTP/1.1 server for JSON-RPC and REST.
// Parity: reference src/httpserver.{h,cpp} (libevent server, -rpcbind/-rpcallowip,
// -rpcthreads workers, -rpcworkqueue depth, -rpcservertimeout, path handlers) and
// src/httprpc.cpp (Basic auth against -rpcuser/-rpcpassword, -rpcauth salted HMAC,
// cookie file; JSON-RPC over POST "/" and "/wallet/<name>"), src/rest.cpp (/rest/*).
//
// Design: an accept thread hands each connection to a bounded pool of connection
// threads (keep-alive, per-request read timeout). Long-poll RPCs therefore do not block
// other clients beyond the -rpcthreads limit, like the reference's work queue.
#pragma once
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace bcp {

struct HTTPRequest {
    std::string method, uri, version, body, peer;
    std::map<std::string, std::string> headers; // lower-case names
    std::string Header(const std::string& name) const {
        auto it = headers.find(name);
        return it == headers.end() ? std::string() : it->second;
    }
};

struct HTTPReply {
    int status = 200;
    std::string contentType = "application/json";
    std::string body;
    std::map<std::string, std::string> extraHeaders;
};

typedef std::function<bool(const HTTPRequest&, HTTPReply&)> HTTPHandler;

class HTTPServer {
public:
    struct Options {
        std::vector<std::pair<std::string, int>> bind; // address, port
        std::vector<std::string> allowSubnets;         // "127.0.0.1", "10.0.0.0/8", "::1"
        int threads = 4;
        int timeoutSeconds = 30;
        int maxConnections = 128;
        int workQueueDepth = 16; // -rpcworkqueue: requests waiting beyond the -rpcthreads running ones
    };
    explicit HTTPServer(const Options& opts);
    ~HTTPServer();
    bool Start(std::string& err);
    void Stop();
    void RegisterHandler(const std::string& prefix, bool exactMatch, HTTPHandler handler);
    void UnregisterHandler(const std::string& prefix);
    int BoundPort() const { return boundPort; }

private:
    void AcceptLoop(int fd);
    void ServeConnection(int fd, std::string peer);
    bool Allowed(const std::string& peer) const;
    std::atomic<int> inFlight{0}; // requests being dispatched
    bool Dispatch(const HTTPRequest& req, HTTPReply& rep);

    Options opts;
    std::vector<int> listenFds;
    std::vector<std::thread> acceptThreads;
    std::atomic<bool> stopping{false};
    std::atomic<int> activeConns{0};
    std::mutex csHandlers;
    std::vector<std::tuple<std::string, bool, HTTPHandler>> handlers;
    std::mutex csConns;
    std::vector<int> connFds;
    int boundPort = 0;
};

// JSON-RPC endpoint with authentication (httprpc.cpp).
bool StartHTTPRPC(HTTPServer& server, const std::string& datadir, std::string& err);
void StopHTTPRPC(const std::string& datadir);
// REST endpoints (rest.cpp).
void StartREST(HTTPServer& server);
// Browser wallet GUI at GET /gui (webgui.cpp), behind the RPC credentials.
void StartWebGUI(HTTPServer& server);
bool RPCAuthorizedHeader(const std::string& authorization, std::string& user);

// Minimal blocking HTTP client (bcp-cli, tests).
bool HTTPPost(const std::string& host, int port, const std::string& path, const std::string& auth,
              const std::string& body, int& status, std::string& response, int timeoutSeconds = 900);

} // namespace bcp
