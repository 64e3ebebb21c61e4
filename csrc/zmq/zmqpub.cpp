#include "zmq/zmqpub.h"
#include "consensus/chain.h"
#include "net/netaddress.h"
#include "node/node.h"
#include "primitives/block.h"
#include "util/util.h"

#include <fcntl.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>

namespace bcp {

// ------------------------------------------------------------------ ZMTP framing
static std::string Greeting() {
    std::string g(64, '\0');
    g[0] = (char)0xFF;
    g[9] = 0x7F;
    g[10] = 3; // ZMTP 3.0
    g[11] = 0;
    memcpy(&g[12], "NULL", 4);
    g[32] = 0; // as-server: unused by NULL
    return g;
}

static void AppendFrame(std::string& out, const std::string& body, bool more, bool command) {
    unsigned char flags = (more ? 0x01 : 0) | (command ? 0x04 : 0);
    if (body.size() > 255) {
        flags |= 0x02;
        out.push_back((char)flags);
        for (int i = 7; i >= 0; i--) out.push_back((char)((uint64_t)body.size() >> (8 * i)));
    } else {
        out.push_back((char)flags);
        out.push_back((char)body.size());
    }
    out += body;
}

static std::string ReadyCommand() {
    std::string body;
    body.push_back(5);
    body += "READY";
    const std::string name = "Socket-Type", value = "PUB";
    body.push_back((char)name.size());
    body += name;
    for (int i = 3; i >= 0; i--) body.push_back((char)(value.size() >> (8 * i)));
    body += value;
    std::string out;
    AppendFrame(out, body, false, true);
    return out;
}

static bool SendAll(int fd, const std::string& s) {
    size_t off = 0;
    while (off < s.size()) {
        struct pollfd p = {fd, POLLOUT, 0};
        if (poll(&p, 1, 2000) <= 0) return false;
        const ssize_t n = send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
        if (n <= 0) {
            if (n < 0 && (errno == EINTR || errno == EAGAIN)) continue;
            return false;
        }
        off += (size_t)n;
    }
    return true;
}

bool ZmtpPublisher::Start(std::string& err) {
    // tcp://host:port  (host "*" = all interfaces)
    const std::string prefix = "tcp://";
    if (endpoint.compare(0, prefix.size(), prefix) != 0) {
        err = "Only tcp:// ZMQ endpoints are supported: " + endpoint;
        return false;
    }
    std::string hostport = endpoint.substr(prefix.size());
    int p = 0;
    std::string host;
    SplitHostPort(hostport, p, host);
    if (host == "*" || host.empty()) host = "0.0.0.0";
    CService svc;
    if (!Lookup(host, svc, p, false) || p == 0) {
        err = "Invalid ZMQ endpoint: " + endpoint;
        return false;
    }
    struct sockaddr_storage ss;
    socklen_t len = sizeof(ss);
    svc.GetSockAddr((struct sockaddr*)&ss, &len);
    listenFd = socket(((struct sockaddr*)&ss)->sa_family, SOCK_STREAM, IPPROTO_TCP);
    int one = 1;
    setsockopt(listenFd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (listenFd < 0 || bind(listenFd, (struct sockaddr*)&ss, len) != 0 || listen(listenFd, 64) != 0) {
        err = "Failed to bind ZMQ address " + endpoint + ": " + strerror(errno);
        if (listenFd >= 0) close(listenFd);
        listenFd = -1;
        return false;
    }
    port = p;
    th = std::thread([this] {
        RenameThread("bcp-zmq");
        Loop();
    });
    return true;
}

void ZmtpPublisher::Stop() {
    stop = true;
    if (th.joinable()) th.join();
    std::lock_guard<std::mutex> l(cs);
    for (auto& p : peers) close(p->fd);
    peers.clear();
    if (listenFd >= 0) close(listenFd);
    listenFd = -1;
}

size_t ZmtpPublisher::SubscriberCount() {
    std::lock_guard<std::mutex> l(cs);
    size_t n = 0;
    for (auto& p : peers) n += p->ready && !p->subs.empty();
    return n;
}

bool ZmtpPublisher::HandleInput(Peer& p) {
    // greeting (64 bytes) then frames
    if (!p.ready) {
        if (p.inbuf.size() < 64) return true;
        if ((unsigned char)p.inbuf[0] != 0xFF || p.inbuf[9] != 0x7F || p.inbuf[10] < 3) return false;
        p.inbuf.erase(0, 64);
        p.ready = true;
    }
    for (;;) {
        if (p.inbuf.size() < 2) return true;
        const unsigned char flags = (unsigned char)p.inbuf[0];
        size_t hdr = 2;
        uint64_t size = (unsigned char)p.inbuf[1];
        if (flags & 0x02) {
            if (p.inbuf.size() < 9) return true;
            size = 0;
            for (int i = 1; i <= 8; i++) size = (size << 8) | (unsigned char)p.inbuf[i];
            hdr = 9;
        }
        if (size > (1 << 20)) return false;
        if (p.inbuf.size() < hdr + size) return true;
        const std::string body = p.inbuf.substr(hdr, (size_t)size);
        p.inbuf.erase(0, hdr + (size_t)size);
        if (flags & 0x04) {
            // command: READY (ignored), SUBSCRIBE / CANCEL (ZMTP 3.1)
            if (body.empty()) continue;
            const size_t nlen = (unsigned char)body[0];
            const std::string name = body.substr(1, nlen);
            const std::string data = body.substr(1 + nlen);
            if (name == "SUBSCRIBE") p.subs.insert(data);
            else if (name == "CANCEL") {
                auto it = p.subs.find(data);
                if (it != p.subs.end()) p.subs.erase(it);
            }
        } else if (!body.empty()) {
            // ZMTP 3.0 subscription message: 0x01 topic / 0x00 topic
            if (body[0] == 1) p.subs.insert(body.substr(1));
            else if (body[0] == 0) {
                auto it = p.subs.find(body.substr(1));
                if (it != p.subs.end()) p.subs.erase(it);
            }
        }
    }
}

void ZmtpPublisher::Loop() {
    const std::string greet = Greeting() + ReadyCommand();
    while (!stop) {
        std::vector<struct pollfd> fds;
        fds.push_back({listenFd, POLLIN, 0});
        {
            std::lock_guard<std::mutex> l(cs);
            for (auto& p : peers) fds.push_back({p->fd, POLLIN, 0});
        }
        if (poll(fds.data(), fds.size(), 100) <= 0) continue;
        if (fds[0].revents & POLLIN) {
            const int fd = accept(listenFd, nullptr, nullptr);
            if (fd >= 0) {
                int one = 1;
                setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
                if (SendAll(fd, greet)) {
                    std::lock_guard<std::mutex> l(cs);
                    peers.emplace_back(new Peer{fd});
                } else {
                    close(fd);
                }
            }
        }
        std::lock_guard<std::mutex> l(cs);
        for (size_t i = 1; i < fds.size(); i++) {
            if (!(fds[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
            auto it = std::find_if(peers.begin(), peers.end(), [&](const std::unique_ptr<Peer>& p) { return p->fd == fds[i].fd; });
            if (it == peers.end()) continue;
            char buf[4096];
            const ssize_t n = recv(fds[i].fd, buf, sizeof(buf), MSG_DONTWAIT);
            bool keep = n > 0;
            if (keep) {
                (*it)->inbuf.append(buf, (size_t)n);
                keep = HandleInput(**it);
            } else if (n < 0 && (errno == EAGAIN || errno == EINTR)) {
                keep = true;
            }
            if (!keep) {
                close((*it)->fd);
                peers.erase(it);
            }
        }
    }
}

void ZmtpPublisher::Publish(const std::vector<std::string>& frames) {
    std::string wire;
    for (size_t i = 0; i < frames.size(); i++) AppendFrame(wire, frames[i], i + 1 < frames.size(), false);
    std::lock_guard<std::mutex> l(cs);
    for (auto it = peers.begin(); it != peers.end();) {
        Peer& p = **it;
        bool match = false;
        for (const std::string& s : p.subs)
            if (frames[0].compare(0, s.size(), s) == 0) {
                match = true;
                break;
            }
        if (p.ready && match && !SendAll(p.fd, wire)) {
            close(p.fd);
            it = peers.erase(it);
            continue;
        }
        ++it;
    }
}

// ------------------------------------------------------------------ notifier
bool ZMQNotifier::Init(std::string& err) {
    static const char* kTypes[] = {"hashblock", "hashtx", "rawblock", "rawtx"};
    for (const char* t : kTypes) {
        const std::string arg = std::string("-zmqpub") + t;
        if (!gArgs.IsArgSet(arg)) continue;
        const std::string ep = gArgs.GetArg(arg, "");
        auto it = publishers.find(ep);
        if (it == publishers.end()) {
            std::unique_ptr<ZmtpPublisher> pub(new ZmtpPublisher(ep));
            if (!pub->Start(err)) return false;
            it = publishers.emplace(ep, std::move(pub)).first;
        }
        notifiers.push_back({t, it->second.get(), 0});
        LogPrintf("zmq: Outbound message high water mark for %s at %s\n", t, ep.c_str());
    }
    return true;
}

void ZMQNotifier::Shutdown() {
    std::lock_guard<std::mutex> l(cs);
    notifiers.clear();
    publishers.clear();
}

std::vector<std::pair<std::string, std::string>> ZMQNotifier::ActiveNotifiers() const {
    std::vector<std::pair<std::string, std::string>> r;
    for (const Notifier& n : notifiers) r.push_back({n.type, n.pub->Endpoint()});
    return r;
}

void ZMQNotifier::Send(Notifier& n, const std::string& payload) {
    unsigned char seq[4];
    for (int i = 0; i < 4; i++) seq[i] = (unsigned char)(n.nSequence >> (8 * i));
    n.pub->Publish({n.type, payload, std::string((const char*)seq, 4)});
    n.nSequence++;
}

static std::string ReversedHash(const uint256& h) {
    std::string s(h.begin(), h.end());
    std::reverse(s.begin(), s.end());
    return s;
}

void ZMQNotifier::UpdatedBlockTip(const CBlockIndex* pindexNew, const CBlockIndex* pindexFork, bool fInitialDownload) {
    if (fInitialDownload || pindexNew == pindexFork) return;
    std::lock_guard<std::mutex> l(cs);
    for (Notifier& n : notifiers) {
        if (n.type == "hashblock") {
            Send(n, ReversedHash(pindexNew->GetBlockHash()));
        } else if (n.type == "rawblock") {
            NodeContext* node = GetNode();
            CBlock block;
            if (!node || !node->chainstate || !node->chainstate->ReadBlock(block, pindexNew, false)) continue;
            const std::vector<unsigned char> raw = SerializeToBytes(block);
            Send(n, std::string(raw.begin(), raw.end()));
        }
    }
}

void ZMQNotifier::NotifyTx(const CTransaction& tx) {
    std::lock_guard<std::mutex> l(cs);
    for (Notifier& n : notifiers) {
        if (n.type == "hashtx") {
            Send(n, ReversedHash(tx.GetHash()));
        } else if (n.type == "rawtx") {
            const std::vector<unsigned char> raw = SerializeToBytes(tx);
            Send(n, std::string(raw.begin(), raw.end()));
        }
    }
}

void ZMQNotifier::TransactionAddedToMempool(const CTransactionRef& tx) { NotifyTx(*tx); }

void ZMQNotifier::BlockConnected(const std::shared_ptr<const CBlock>& block, const CBlockIndex*,
                                 const std::vector<CTransactionRef>&) {
    for (const CTransactionRef& tx : block->vtx) NotifyTx(*tx);
}

void ZMQNotifier::BlockDisconnected(const std::shared_ptr<const CBlock>& block) {
    for (const CTransactionRef& tx : block->vtx) NotifyTx(*tx);
}

// ------------------------------------------------------------------ init hooks
static std::unique_ptr<ZMQNotifier> g_zmq;

bool StartZMQ(NodeContext& node, std::string& err) {
    std::unique_ptr<ZMQNotifier> z(new ZMQNotifier());
    if (!z->Init(err)) return false;
    if (!z->Active()) return true;
    GetMainSignals().Register(z.get());
    node.zmq = z.get();
    g_zmq = std::move(z);
    return true;
}

void StopZMQ(NodeContext& node) {
    if (!g_zmq) return;
    GetMainSignals().Unregister(g_zmq.get());
    g_zmq->Shutdown();
    node.zmq = nullptr;
    g_zmq.reset();
}

} // namespace bcp
