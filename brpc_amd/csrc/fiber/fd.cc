// fd waiting for fibers (role of bthread/fd.cpp:111-558): each fd owns a
// butex; a dedicated epoll pthread bumps and wakes it with EPOLLONESHOT
// registrations. Used by fiber::connect and by code that needs to block on a
// raw fd (pipes, eventfds) without occupying a worker.
#include <fcntl.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <mutex>
#include <thread>

#include "base/logging.h"
#include "base/time.h"
#include "fiber/butex.h"
#include "fiber/internal.h"

namespace mrpc {
namespace fiber {

namespace {
const int kBlockShift = 12;
const int kBlockSize = 1 << kBlockShift;
const int kMaxBlocks = 1 << 10;  // 4M fds

class EpollThread {
public:
    EpollThread() : _epfd(-1) {}
    int start() {
        std::lock_guard<std::mutex> g(_mu);
        if (_epfd >= 0) return 0;
        _epfd = epoll_create1(EPOLL_CLOEXEC);
        if (_epfd < 0) return -1;
        for (int i = 0; i < kMaxBlocks; ++i) _blocks[i].store(nullptr, std::memory_order_relaxed);
        std::thread([this] { run(); }).detach();
        return 0;
    }
    std::atomic<int>* get_butex(int fd, bool create) {
        if (fd < 0) return nullptr;
        int bi = fd >> kBlockShift;
        if (bi >= kMaxBlocks) return nullptr;
        auto* blk = _blocks[bi].load(std::memory_order_acquire);
        if (!blk) {
            if (!create) return nullptr;
            auto* nb = new std::atomic<std::atomic<int>*>[kBlockSize];
            for (int i = 0; i < kBlockSize; ++i) nb[i].store(nullptr, std::memory_order_relaxed);
            std::atomic<std::atomic<int>*>* expected = nullptr;
            if (!_blocks[bi].compare_exchange_strong(expected, nb)) {
                delete[] nb;
                blk = expected;
            } else {
                blk = nb;
            }
        }
        auto& slot = blk[fd & (kBlockSize - 1)];
        std::atomic<int>* b = slot.load(std::memory_order_acquire);
        if (!b && create) {
            std::atomic<int>* nb = butex_create();
            std::atomic<int>* expected = nullptr;
            if (slot.compare_exchange_strong(expected, nb)) {
                b = nb;
            } else {
                butex_destroy(nb);
                b = expected;
            }
        }
        return b;
    }
    int wait(int fd, unsigned events, const timespec* abstime) {
        if (start() != 0) return -1;
        std::atomic<int>* b = get_butex(fd, true);
        if (!b) {
            errno = EINVAL;
            return -1;
        }
        const int expected = b->load(std::memory_order_acquire);
        epoll_event ev;
        ev.events = events | EPOLLONESHOT;
        ev.data.fd = fd;
        if (epoll_ctl(_epfd, EPOLL_CTL_ADD, fd, &ev) != 0) {
            if (errno != EEXIST || epoll_ctl(_epfd, EPOLL_CTL_MOD, fd, &ev) != 0) return -1;
        }
        while (b->load(std::memory_order_acquire) == expected) {
            if (butex_wait(b, expected, abstime) < 0) {
                if (errno == EWOULDBLOCK) break;
                if (errno == ETIMEDOUT || errno == EINTR || errno == ESTOP) {
                    int e = errno;
                    epoll_ctl(_epfd, EPOLL_CTL_DEL, fd, nullptr);
                    errno = e;
                    return -1;
                }
            }
        }
        return 0;
    }
    int close_fd(int fd) {
        std::atomic<int>* b = get_butex(fd, false);
        if (b && _epfd >= 0) {
            epoll_ctl(_epfd, EPOLL_CTL_DEL, fd, nullptr);
            b->fetch_add(1, std::memory_order_release);
            butex_wake_all(b);
        }
        return ::close(fd);
    }

private:
    void run() {
        pthread_setname_np(pthread_self(), "mrpc_fdwait");
        epoll_event evs[64];
        for (;;) {
            int n = epoll_wait(_epfd, evs, 64, -1);
            if (n < 0) {
                if (errno == EINTR) continue;
                PLOG(ERROR) << "epoll_wait";
                break;
            }
            for (int i = 0; i < n; ++i) {
                std::atomic<int>* b = get_butex(evs[i].data.fd, false);
                if (b) {
                    b->fetch_add(1, std::memory_order_release);
                    butex_wake_all(b);
                }
            }
        }
    }
    std::mutex _mu;
    int _epfd;
    std::atomic<std::atomic<std::atomic<int>*>*> _blocks[kMaxBlocks];
};

EpollThread& epoll_thread() {
    static EpollThread* t = new EpollThread;
    return *t;
}
}  // namespace

int fd_wait(int fd, unsigned events) { return epoll_thread().wait(fd, events, nullptr); }

int fd_timedwait(int fd, unsigned events, const timespec* abstime) {
    return epoll_thread().wait(fd, events, abstime);
}

int connect(int sockfd, const struct sockaddr* addr, unsigned addrlen, int64_t timeout_ms) {
    int fl = fcntl(sockfd, F_GETFL, 0);
    if (!(fl & O_NONBLOCK)) fcntl(sockfd, F_SETFL, fl | O_NONBLOCK);
    int rc = ::connect(sockfd, addr, addrlen);
    if (rc == 0) return 0;
    if (errno != EINPROGRESS) return -1;
    timespec abst;
    const timespec* pabs = nullptr;
    if (timeout_ms >= 0) {
        abst = realtime_after_us(timeout_ms * 1000);
        pabs = &abst;
    }
    if (fd_timedwait(sockfd, EPOLLOUT, pabs) != 0) return -1;
    int err = 0;
    socklen_t len = sizeof(err);
    if (getsockopt(sockfd, SOL_SOCKET, SO_ERROR, &err, &len) != 0) return -1;
    if (err) {
        errno = err;
        return -1;
    }
    return 0;
}

int close_fd(int fd) { return epoll_thread().close_fd(fd); }

}  // namespace fiber
}  // namespace mrpc
