// RDMA transport: a whole-connection verbs data plane that replaces the TCP
// byte stream after a TCP handshake, with registered-memory Buf blocks and
// credit-based flow control. Capability parity with the reference's
// src/brpc/rdma/ (rdma_endpoint.cpp 79-82/409/552 handshake, 771-895
// CutFromIOBufList with SEND_WITH_IMM + ACK-in-imm sliding window,
// 926 HandleCompletion, 1008 PostRecv, 1317-1342 PollCq; block_pool.cpp
// 8K/64K/2M block types over registered regions; rdma_helper.cpp dlopen'd
// verbs, RegisterMemoryForRdma and the blockmem_allocate swap).
//
// MI355X-first differences:
//  * The verbs layer is a small Provider interface. `ibverbs` (dlopen of
//    libibverbs.so.1, built only where rdma-core headers exist) registers
//    host blocks with ibv_reg_mr and HBM with ibv_reg_dmabuf_mr (GPUDirect:
//    the NIC gathers DEVICE Buf blocks straight out of HBM). `soft` is an
//    in-process RC emulator with identical queue/credit semantics (RNR
//    retry = queue until a recv is posted), so the endpoint logic is tested
//    on machines without an HCA — neither this container nor the MI355X
//    pool has one.
//  * Registered memory is a per-kind pool: 8 KiB Buf blocks (the default
//    Buf allocator is swapped, like blockmem_allocate), 64 KiB and 2 MiB
//    receive blocks, regions grown on demand; DEVICE memory is registered
//    by the user (RegisterMemoryForRdma) and never touched by host code.
//  * Completions are drained by one fiber per endpoint that parks on the
//    CQ's notification fd (fiber::fd_timedwait), so polling never blocks a
//    worker pthread.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "base/buf.h"
#include "fiber/fiber.h"

namespace mrpc {
class Socket;
typedef uint64_t SocketId;

namespace rdma {

// ---------------------------------------------------------------- provider

struct Sge {
    uint64_t addr;
    uint32_t length;
    uint32_t lkey;
};

enum WcOpcode { WC_SEND = 0, WC_RECV = 1 };

struct WorkCompletion {
    uint64_t wr_id = 0;
    int opcode = WC_SEND;
    int status = 0;  // 0 = success
    uint32_t byte_len = 0;
    uint32_t imm = 0;
    bool has_imm = false;
};

// Address of a queue pair: the fields a verbs RC connection needs.
struct QpAddress {
    uint64_t gid_hi = 0, gid_lo = 0;
    uint32_t qpn = 0;
    uint16_t lid = 0;
};

class CompletionQueue {
public:
    virtual ~CompletionQueue() {}
    // Up to n completions; 0 when empty, -1 on error.
    virtual int Poll(WorkCompletion* wc, int n) = 0;
    // Request an event on the next completion (ibv_req_notify_cq).
    virtual int Arm() = 0;
    // Readable when an armed completion arrived; consume with AckEvent().
    virtual int notify_fd() const = 0;
    virtual void AckEvent() = 0;
};

class QueuePair {
public:
    virtual ~QueuePair() {}
    virtual QpAddress local() const = 0;
    // INIT -> RTR -> RTS against the remote address.
    virtual int Connect(const QpAddress& remote) = 0;
    // RESET -> INIT: receives may be posted from here on (verbs refuse them
    // in RESET), before Connect() makes the QP ready to receive and send.
    virtual int Prepare() { return 0; }
    virtual int PostSend(uint64_t wr_id, const Sge* sge, int nsge, bool with_imm, uint32_t imm, bool signaled) = 0;
    virtual int PostRecv(uint64_t wr_id, const Sge& sge) = 0;
};

class Provider {
public:
    virtual ~Provider() {}
    virtual const char* name() const = 0;
    virtual std::string device_name() const = 0;
    virtual int max_sge() const = 0;
    // Register [p, p+n). device=true: HBM (dmabuf path). Returns 0 + lkey.
    virtual int RegisterMemory(void* p, size_t n, bool device, int gpu, uint32_t* lkey) = 0;
    virtual void DeregisterMemory(void* p) = 0;
    virtual std::unique_ptr<CompletionQueue> CreateCq(int depth) = 0;
    virtual std::unique_ptr<QueuePair> CreateQp(CompletionQueue* cq, int sq_depth, int rq_depth) = 0;
};

// Built-in providers (nullptr when unavailable; *why explains).
std::unique_ptr<Provider> CreateSoftProvider();
std::unique_ptr<Provider> CreateIbverbsProvider(std::string* why);
bool IbverbsCompiledIn();

// ---------------------------------------------------------------- global

// Select the provider (-rdma_provider=auto|ibverbs|soft; auto prefers a
// real HCA) and swap the default Buf block allocator to the registered pool.
// Idempotent. Returns 0, or -1 with *err.
int GlobalRdmaInitialize(std::string* err = nullptr);
bool RdmaAvailable();
Provider* GetProvider();

// Register user memory so Buf blocks pointing into it go out zero-copy
// (kind DEVICE = GPUDirect HBM). Returns 0 on success.
int RegisterMemoryForRdma(void* p, size_t n, MemKind kind = MemKind::HOST, int gpu = -1);
void DeregisterMemoryForRdma(void* p);
// lkey of a registered range, false if [p, p+n) is not fully registered.
bool LookupLkey(const void* p, size_t n, uint32_t* lkey);
// HBM -> dmabuf fd export used by the ibverbs provider to register DEVICE
// memory (ibv_reg_dmabuf_mr). Installed by the HIP runtime (gpu/runtime.cc,
// hipMemGetHandleForAddressRange) so this layer never links HIP itself.
using DmabufExportFn = int (*)(void* p, size_t n, int gpu, int* fd, uint64_t* offset);
void SetDmabufExportHook(DmabufExportFn fn);
DmabufExportFn GetDmabufExportHook();

struct PoolStats {
    int64_t regions = 0, region_bytes = 0;
    int64_t blocks_8k = 0, blocks_64k = 0, blocks_2m = 0;  // handed out
    int64_t fallback_allocs = 0;                            // served unregistered
    int64_t user_regions = 0;
};
PoolStats GetPoolStats();
// Allocate / free a registered receive block of one of the pool classes
// (8 KiB, 64 KiB, 2 MiB including the Buf block header).
BufBlock* NewRegisteredBlock(size_t total_bytes);

// ---------------------------------------------------------------- handshake

// Sent by the client right after TCP connect, answered by the server. Fixed
// size, big-endian fields.
struct Hello {
    static const size_t kSize = 44;
    static const uint16_t kVersion = 1;
    uint16_t version = kVersion;
    uint16_t sq_size = 0;
    uint16_t rq_size = 0;
    uint16_t flags = 0;  // bit0: GPUDirect (DEVICE blocks) supported
    uint32_t block_size = 0;  // receive buffer capacity (bytes per message)
    QpAddress addr;
    void Serialize(char* out) const;  // writes kSize bytes incl. "RDMA"
    bool Parse(const char* in);
};
extern const char kMagic[4];

// ---------------------------------------------------------------- endpoint

struct EndpointStats {
    int64_t sent_msgs = 0, sent_bytes = 0, recv_msgs = 0, recv_bytes = 0;
    int64_t pure_acks_sent = 0, bounce_copies = 0, window_full = 0;
};

class Endpoint : public std::enable_shared_from_this<Endpoint> {
public:
    explicit Endpoint(SocketId host);
    ~Endpoint();
    // Create CQ/QP and post the receive ring.
    int Init(std::string* err);
    void FillHello(Hello* h) const;
    // Connect the QP to the peer described by `h` and start polling.
    int Start(const Hello& h, std::string* err);

    // Post the front of `pieces` as SEND_WITH_IMM work requests (zero copy
    // for registered blocks). Bytes consumed, or -1 + EAGAIN when the remote
    // window / send queue is full.
    ssize_t CutFromBufList(Buf* const* pieces, size_t count);
    // Move received bytes into *out. -1 + EAGAIN when nothing is queued.
    ssize_t ReadInto(Buf* out);
    // Park until the window may have opened (or abstime / shutdown).
    int WaitWritable(const timespec* abstime);
    void Shutdown();
    bool started() const { return _started.load(std::memory_order_acquire); }
    EndpointStats stats() const;
    std::string Describe() const;

private:
    static void* PollLoop(void* arg);
    int HandleCompletions();
    int PostRecvSlot(size_t slot);
    int SendPureAckLocked();
    void FailHost(int err, const char* what);

    SocketId _host;
    std::unique_ptr<CompletionQueue> _cq;
    std::unique_ptr<QueuePair> _qp;
    int _sq_size = 0, _rq_size = 0;
    size_t _recv_block_total = 0;  // pool class of receive blocks
    uint32_t _local_block_cap = 0, _remote_block_cap = 0;
    bool _remote_gpudirect = false;

    // send side (guarded by _send_mu)
    std::mutex _send_mu;
    std::vector<Buf> _sbuf;       // payload kept alive until its completion
    uint64_t _sq_posted = 0;      // wr ids handed out
    uint64_t _sq_completed = 0;   // all wr ids < this are complete
    int _unsignaled = 0;
    std::atomic<int> _window{0};  // remote receive credits
    std::atomic<int> _new_acks{0};  // our reposted receives not yet returned
    std::atomic<int>* _write_butex;

    // receive side
    std::vector<BufBlock*> _rbuf;
    std::mutex _in_mu;
    Buf _in;
    std::atomic<bool> _started{false};
    std::atomic<bool> _stop{false};
    fiber::fiber_t _poller = 0;
    bool _poller_running = false;

    mutable std::mutex _stat_mu;
    EndpointStats _stats;
};

// Client side: after TCP connect on a non-blocking fd, exchange hellos and
// bring up the endpoint. Returns the endpoint or nullptr (+ *err).
std::shared_ptr<Endpoint> ClientHandshake(SocketId host, int fd, const timespec* abstime, std::string* err);
// Server side: `in` holds the first bytes of an accepted connection.
// Returns 1 (handshake done, hello consumed, *ep set), 0 (need more bytes),
// -1 (not an RDMA client: plain TCP).
int ServerTryHandshake(SocketId host, int fd, Buf* in, std::shared_ptr<Endpoint>* ep, std::string* err);

// rdma_performance-style numbers and /rdma builtin page.
std::string DescribeRdma();

}  // namespace rdma
}  // namespace mrpc
