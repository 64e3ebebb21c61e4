// ZeroMQ-compatible block/transaction notifications.
// Parity: reference src/zmq/zmqnotificationinterface.{h,cpp} and zmqpublishnotifier.cpp:
// -zmqpubhashblock / -zmqpubhashtx / -zmqpubrawblock / -zmqpubrawtx=<tcp://addr:port>,
// three-part messages [topic, payload, LE32 sequence], per-notifier sequence counters,
// notifiers sharing one PUB socket per address, block notifications skipped in IBD.
//
// libzmq is not available on this platform, so the PUB side of ZMTP/3.0 (NULL security
// mechanism, READY handshake, SUBSCRIBE/CANCEL as 0x01/0x00-prefixed frames or 3.1
// commands, prefix topic matching) is implemented natively over POSIX sockets. Standard
// ZMQ SUB sockets (libzmq, pyzmq) interoperate with it.
#pragma once
#include "node/signals.h"

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace bcp {

class ZmtpPublisher {
public:
    explicit ZmtpPublisher(const std::string& endpoint) : endpoint(endpoint) {}
    ~ZmtpPublisher() { Stop(); }
    bool Start(std::string& err);
    void Stop();
    // Send a multipart message to every subscriber whose subscription prefixes frames[0].
    void Publish(const std::vector<std::string>& frames);
    const std::string& Endpoint() const { return endpoint; }
    int BoundPort() const { return port; }
    size_t SubscriberCount();

private:
    struct Peer {
        int fd;
        bool ready = false;
        std::string inbuf;
        std::multiset<std::string> subs;
    };
    void Loop();
    bool HandleInput(Peer& p);

    std::string endpoint;
    int listenFd = -1;
    int port = 0;
    std::atomic<bool> stop{false};
    std::thread th;
    std::mutex cs;
    std::vector<std::unique_ptr<Peer>> peers;
};

class ZMQNotifier : public CValidationInterface {
public:
    // Parse -zmqpub* arguments; returns false on a bad endpoint.
    bool Init(std::string& err);
    void Shutdown();
    bool Active() const { return !notifiers.empty(); }
    std::vector<std::pair<std::string, std::string>> ActiveNotifiers() const; // (type, endpoint)

    void UpdatedBlockTip(const CBlockIndex* pindexNew, const CBlockIndex* pindexFork, bool fInitialDownload) override;
    void TransactionAddedToMempool(const CTransactionRef& tx) override;
    void BlockConnected(const std::shared_ptr<const CBlock>& block, const CBlockIndex* pindex,
                        const std::vector<CTransactionRef>& txnConflicted) override;
    void BlockDisconnected(const std::shared_ptr<const CBlock>& block) override;

private:
    struct Notifier {
        std::string type; // hashblock | hashtx | rawblock | rawtx
        ZmtpPublisher* pub;
        uint32_t nSequence = 0;
    };
    void Send(Notifier& n, const std::string& payload);
    void NotifyTx(const CTransaction& tx);
    std::mutex cs;
    std::map<std::string, std::unique_ptr<ZmtpPublisher>> publishers; // by endpoint
    std::vector<Notifier> notifiers;
};

} // namespace bcp
