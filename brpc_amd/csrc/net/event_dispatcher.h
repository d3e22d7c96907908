// Edge-triggered epoll dispatcher running inside a fiber (role of
// src/brpc/event_dispatcher_epoll.cpp:114-239). On EPOLLIN it calls
// Socket::StartInputEvent which start_urgent()s the reader fiber on this
// worker while the dispatcher fiber is re-queued for other workers to steal,
// keeping the read on the core that took the interrupt.
#pragma once

#include <atomic>

#include <cstdint>

#include "net/socket.h"

namespace mrpc {

class EventDispatcher {
public:
    EventDispatcher();
    ~EventDispatcher();
    int Start();
    bool Running() const;
    // Edge-triggered EPOLLIN consumer for socket_id.
    int AddConsumer(SocketId socket_id, int fd);
    int RemoveConsumer(int fd);
    // Temporarily add EPOLLOUT (one-shot style, via MOD).
    int AddEpollOut(SocketId socket_id, int fd, bool pollin);
    int RemoveEpollOut(SocketId socket_id, int fd, bool pollin);
    void Stop();
    void Join();

private:
    static void* RunThis(void* arg);
    void Run();
    int _epfd;
    int _wakeup_fds[2];
    std::atomic<bool> _stop;
    fiber::fiber_t _tid;
};

EventDispatcher& GetGlobalEventDispatcher(int fd);
int GetEventDispatcherNum();

}  // namespace mrpc
