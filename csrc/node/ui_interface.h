// User-facing notification bus.
// Parity: reference src/ui_interface.h:24 (CClientUIInterface: ThreadSafeMessageBox,
// ThreadSafeQuestion, InitMessage, NotifyNumConnectionsChanged,
// NotifyNetworkActiveChanged, NotifyAlertChanged, LoadWallet, ShowProgress,
// NotifyBlockTip, NotifyHeaderTip, BannedListChanged; message-box style flags) and
// src/noui.cpp (headless sinks: message boxes go to stderr + the log, init messages to
// the log). The reference routes these through boost::signals2; here each signal is a
// small slot list with integer connection handles and a snapshot-then-call emit, so a
// slot may disconnect itself and emits never hold the list lock while running slots.
#pragma once
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace bcp {

class CBlockIndex;

template <typename R, typename... A> class UISignal;

template <typename R, typename... A> class UISignal<R(A...)> {
public:
    using Slot = std::function<R(A...)>;
    int connect(Slot f) {
        std::lock_guard<std::mutex> l(m);
        slots.emplace_back(++nextId, std::move(f));
        return nextId;
    }
    void disconnect(int id) {
        std::lock_guard<std::mutex> l(m);
        for (size_t i = 0; i < slots.size(); ++i)
            if (slots[i].first == id) {
                slots.erase(slots.begin() + i);
                return;
            }
    }
    void disconnect_all() {
        std::lock_guard<std::mutex> l(m);
        slots.clear();
    }
    size_t num_slots() const {
        std::lock_guard<std::mutex> l(m);
        return slots.size();
    }
    // Calls every slot; for bool-returning signals the result is the AND of all
    // slots (true with no slots), matching the reference's boolean combiner.
    R operator()(A... args) const {
        std::vector<std::pair<int, Slot>> snap;
        {
            std::lock_guard<std::mutex> l(m);
            snap = slots;
        }
        if constexpr (std::is_same<R, bool>::value) {
            bool r = true;
            for (auto& s : snap) r = s.second(args...) && r;
            return r;
        } else {
            for (auto& s : snap) s.second(args...);
        }
    }

private:
    mutable std::mutex m;
    std::vector<std::pair<int, Slot>> slots;
    int nextId = 0;
};

class CWallet;

class CClientUIInterface {
public:
    enum MessageBoxFlags : unsigned {
        ICON_INFORMATION = 0,
        ICON_WARNING = (1U << 0),
        ICON_ERROR = (1U << 1),
        ICON_MASK = (ICON_INFORMATION | ICON_WARNING | ICON_ERROR),
        BTN_OK = 0x00000400U,
        BTN_YES = 0x00004000U,
        BTN_NO = 0x00010000U,
        BTN_ABORT = 0x00040000U,
        BTN_RETRY = 0x00080000U,
        BTN_IGNORE = 0x00100000U,
        BTN_CLOSE = 0x08000000U,
        BTN_CANCEL = 0x00400000U,
        BTN_MASK = (BTN_OK | BTN_YES | BTN_NO | BTN_ABORT | BTN_RETRY | BTN_IGNORE | BTN_CLOSE | BTN_CANCEL),
        MODAL = 0x10000000U,
        SECURE = 0x40000000U,
        MSG_INFORMATION = ICON_INFORMATION,
        MSG_WARNING = (ICON_WARNING | BTN_OK | MODAL),
        MSG_ERROR = (ICON_ERROR | BTN_OK | MODAL)
    };
    enum ChangeType { CT_NEW, CT_UPDATED, CT_DELETED };

    UISignal<bool(const std::string& message, const std::string& caption, unsigned style)> ThreadSafeMessageBox;
    UISignal<bool(const std::string& message, const std::string& noninteractive, const std::string& caption,
                  unsigned style)>
        ThreadSafeQuestion;
    UISignal<void(const std::string& message)> InitMessage;
    UISignal<void(int newNumConnections)> NotifyNumConnectionsChanged;
    UISignal<void(bool networkActive)> NotifyNetworkActiveChanged;
    UISignal<void()> NotifyAlertChanged;
    UISignal<void(CWallet* wallet)> LoadWallet;
    UISignal<void(const std::string& title, int nProgress)> ShowProgress;
    UISignal<void(bool fInitialDownload, const CBlockIndex* newTip)> NotifyBlockTip;
    UISignal<void(bool fInitialDownload, const CBlockIndex* newTip)> NotifyHeaderTip;
    UISignal<void()> BannedListChanged;
};

extern CClientUIInterface uiInterface;

// Headless sinks (reference noui.cpp): connect once per process; returns false if
// already connected.
bool noui_connect();
void noui_disconnect();

// Report an error / warning through ThreadSafeMessageBox (reference InitError/InitWarning).
bool InitError(const std::string& str);
void InitWarning(const std::string& str);

} // namespace bcp
