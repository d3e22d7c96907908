#include "net/event_dispatcher.h"

#include <fcntl.h>
#include <sys/epoll.h>
#include <unistd.h>

#include <time.h>

#include <cerrno>
#include <mutex>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "base/tsan.h"
#include "fiber/fiber.h"

DEFINE_int32(event_dispatcher_num, 1, "Number of event dispatchers");
DEFINE_int32(event_dispatcher_spin_us, 0,
             "after handling events, poll epoll without blocking for this long before sleeping (0 disables)");
DEFINE_int32(event_dispatcher_nap_us, 50,
             "after the spin window, wait in epoll with this timeout (us) instead of blocking for good, so the "
             "core only ever enters shallow idle states and wakes in a few us (0 disables)");
DEFINE_int32(event_dispatcher_nap_window_ms, 1000,
             "how long after the last event the dispatcher keeps napping before it blocks without a timeout");

namespace mrpc {

EventDispatcher::EventDispatcher() : _epfd(-1), _stop(false), _tid(0) {
    _wakeup_fds[0] = _wakeup_fds[1] = -1;
    _epfd = epoll_create1(EPOLL_CLOEXEC);
    if (_epfd < 0) PLOG(FATAL) << "epoll_create1";
}

EventDispatcher::~EventDispatcher() {
    Stop();
    Join();
    if (_epfd >= 0) close(_epfd);
}

int EventDispatcher::Start() {
    if (_tid) return 0;
    fiber::Attr attr = fiber::ATTR_NORMAL;
    // The dispatcher blocks its worker in epoll_wait; run it as a normal
    // fiber so that start_urgent() hand-offs work as described above.
    if (fiber::start_background(&_tid, &attr, RunThis, this) != 0) {
        LOG(FATAL) << "Fail to start EventDispatcher fiber";
        return -1;
    }
    return 0;
}

bool EventDispatcher::Running() const { return !_stop && _tid != 0; }

void EventDispatcher::Stop() {
    _stop = true;
    if (_epfd >= 0 && _wakeup_fds[1] < 0) {
        if (pipe2(_wakeup_fds, O_CLOEXEC) == 0) {
            epoll_event evt;
            evt.events = EPOLLOUT;
            evt.data.u64 = INVALID_SOCKET_ID;
            epoll_ctl(_epfd, EPOLL_CTL_ADD, _wakeup_fds[1], &evt);
        }
    }
}

void EventDispatcher::Join() {
    if (_tid) {
        fiber::join(_tid);
        _tid = 0;
    }
}

int EventDispatcher::AddConsumer(SocketId socket_id, int fd) {
    epoll_event evt;
    evt.events = EPOLLIN | EPOLLET | EPOLLRDHUP;
    evt.data.u64 = socket_id;
    // epoll_ctl/epoll_pwait2 order the socket's setup before its first
    // event; tell TSan (it does not intercept epoll_pwait2)
    MRPC_TSAN_RELEASE(&_epfd);
    const int rc = epoll_ctl(_epfd, EPOLL_CTL_ADD, fd, &evt);
    MRPC_TSAN_RELEASE(&_epfd);  // and the fd access of epoll_ctl before a close after the first event
    return rc;
}

int EventDispatcher::RemoveConsumer(int fd) {
    if (fd < 0) return -1;
    return epoll_ctl(_epfd, EPOLL_CTL_DEL, fd, nullptr);
}

int EventDispatcher::AddEpollOut(SocketId socket_id, int fd, bool pollin) {
    epoll_event evt;
    evt.data.u64 = socket_id;
    evt.events = EPOLLOUT | EPOLLET;
    MRPC_TSAN_RELEASE(&_epfd);
    if (pollin) {
        evt.events |= EPOLLIN | EPOLLRDHUP;
        return epoll_ctl(_epfd, EPOLL_CTL_MOD, fd, &evt);
    }
    if (epoll_ctl(_epfd, EPOLL_CTL_ADD, fd, &evt) < 0 && errno != EEXIST) return -1;
    return 0;
}

int EventDispatcher::RemoveEpollOut(SocketId socket_id, int fd, bool pollin) {
    if (pollin) {
        epoll_event evt;
        evt.data.u64 = socket_id;
        evt.events = EPOLLIN | EPOLLET | EPOLLRDHUP;
        return epoll_ctl(_epfd, EPOLL_CTL_MOD, fd, &evt);
    }
    return epoll_ctl(_epfd, EPOLL_CTL_DEL, fd, nullptr);
}

void* EventDispatcher::RunThis(void* arg) {
    static_cast<EventDispatcher*>(arg)->Run();
    return nullptr;
}

void EventDispatcher::Run() {
    epoll_event e[32];
    int64_t last_event_ns = 0;
    bool nap_ok = true;  // epoll_pwait2 exists (Linux >= 5.11)
    while (!_stop) {
        int n;
        const int64_t idle_ns = monotonic_ns() - last_event_ns;
        if (FLAGS_event_dispatcher_spin_us > 0 && idle_ns < (int64_t)FLAGS_event_dispatcher_spin_us * 1000) {
            // Right after events the reply of what was just sent usually
            // follows within µs: poll instead of sleeping in the kernel, and
            // yield between polls so fibers queued on this worker still run.
            n = epoll_wait(_epfd, e, 32, 0);
            if (n == 0) {
                fiber::yield();
                continue;
            }
        } else if (nap_ok && FLAGS_event_dispatcher_nap_us > 0 &&
                   idle_ns < (int64_t)FLAGS_event_dispatcher_nap_window_ms * 1000000) {
            // Napping: a blocked core drops into the deepest idle state (100 us
            // exit latency on the MI355X hosts' EPYCs, measured p99 192 us per
            // wake by benchmarks/wake_latency.cc); a core that wakes every
            // ~50 us stays shallow and answers an event in a few us, for ~2%
            // of a core.
            const timespec ts{0, (long)FLAGS_event_dispatcher_nap_us * 1000};
            n = epoll_pwait2(_epfd, e, 32, &ts, nullptr);
            if (n < 0 && errno == ENOSYS) {
                nap_ok = false;
                continue;
            }
            if (n == 0) {
                fiber::yield();
                continue;
            }
        } else {
            n = epoll_wait(_epfd, e, 32, -1);
        }
        if (_stop) break;
        if (n > 0) {
            last_event_ns = monotonic_ns();
            MRPC_TSAN_ACQUIRE(&_epfd);
        }
        if (n < 0) {
            if (errno == EINTR) continue;
            PLOG(ERROR) << "epoll_wait";
            break;
        }
        for (int i = 0; i < n; ++i) {
            if (e[i].data.u64 == INVALID_SOCKET_ID) continue;
            if (e[i].events & (EPOLLIN | EPOLLERR | EPOLLHUP | EPOLLRDHUP)) {
                Socket::StartInputEvent(e[i].data.u64, e[i].events);
            }
        }
        for (int i = 0; i < n; ++i) {
            if (e[i].data.u64 == INVALID_SOCKET_ID) continue;
            if (e[i].events & (EPOLLOUT | EPOLLERR | EPOLLHUP)) Socket::HandleEpollOut(e[i].data.u64);
        }
    }
}

namespace {
std::once_flag g_disp_once;
EventDispatcher* g_disps = nullptr;
int g_ndisp = 1;
}  // namespace

int GetEventDispatcherNum() { return g_ndisp; }

EventDispatcher& GetGlobalEventDispatcher(int fd) {
    std::call_once(g_disp_once, [] {
        g_ndisp = FLAGS_event_dispatcher_num > 0 ? FLAGS_event_dispatcher_num : 1;
        g_disps = new EventDispatcher[g_ndisp];
        for (int i = 0; i < g_ndisp; ++i) g_disps[i].Start();
    });
    if (g_ndisp == 1) return g_disps[0];
    return g_disps[(unsigned)fd % (unsigned)g_ndisp];
}

}  // namespace mrpc
