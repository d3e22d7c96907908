// Combo channels (role of the reference's src/brpc/parallel_channel.h,
// partition_channel.h:30-174, selective_channel.h):
//
//  * ParallelChannel   — fan one call out to N sub channels (CallMapper
//                        maps/splits the request, ResponseMerger reduces),
//                        finish on fail_limit / success_limit. The DP / TP
//                        analog of SURVEY §2.10: on a node each sub channel
//                        can be the xGMI-direct channel to one peer GPU.
//  * PartitionChannel  — a ParallelChannel whose sub channels are the
//                        partitions "i/N" of one naming service (sharding,
//                        the EP analog).
//  * DynamicPartitionChannel — several partitioning schemes at once (N
//                        changes while servers migrate); traffic is split
//                        by the capacity of each scheme.
//  * SelectiveChannel  — load balancing across whole sub channels (replica
//                        groups) with retry on another group and backup
//                        requests.
#pragma once

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "cluster/naming_service.h"
#include "rpc/channel.h"

namespace mrpc {

enum ChannelOwnership { OWNS_CHANNEL, DOESNT_OWN_CHANNEL };

// What one sub channel receives.
struct SubCall {
    enum Flags { DELETE_REQUEST = 1, DELETE_RESPONSE = 2, SKIP = 4, BAD = 8 };
    SubCall() {}
    SubCall(const pb::MethodDescriptor* m, const pb::Message* req, pb::Message* res, int f)
        : method(m), request(req), response(res), flags(f) {}
    static SubCall Skip() { return SubCall(nullptr, nullptr, nullptr, SKIP); }
    static SubCall Bad() { return SubCall(nullptr, nullptr, nullptr, BAD); }
    bool is_skip() const { return flags & SKIP; }
    bool is_bad() const { return flags & BAD; }
    const pb::MethodDescriptor* method = nullptr;
    const pb::Message* request = nullptr;
    pb::Message* response = nullptr;
    int flags = 0;
};

class CallMapper {
public:
    virtual ~CallMapper() {}
    virtual SubCall Map(int channel_index, int channel_count, const pb::MethodDescriptor* method,
                        const pb::Message* request, pb::Message* response) = 0;
    // The part of the parent's request attachment sub call `channel_index`
    // carries. Default: all of it (broadcast). `out` shares the blocks — a
    // slice of an HBM attachment is lent to its peer GPU without a copy.
    virtual void MapAttachment(int channel_index, int channel_count, const Buf& attachment, Buf* out) {
        (void)channel_index;
        (void)channel_count;
        out->append(attachment);
    }
};

// Tensor-parallel style scatter (SURVEY §2.10 TP analog): every sub call
// gets the same request message and the channel_index-th of channel_count
// near-equal contiguous slices of the attachment; the default merge
// appends the sub responses' attachments in channel order, so an echo
// service gathers the original attachment back.
class ScatterAttachmentMapper : public CallMapper {
public:
    SubCall Map(int, int, const pb::MethodDescriptor* method, const pb::Message* request,
                pb::Message* response) override {
        return SubCall(method, request, response ? response->New() : nullptr, SubCall::DELETE_RESPONSE);
    }
    void MapAttachment(int i, int n, const Buf& attachment, Buf* out) override {
        const size_t total = attachment.size();
        const size_t begin = total * (size_t)i / (size_t)n, end = total * (size_t)(i + 1) / (size_t)n;
        Buf view(attachment);  // shares blocks
        view.pop_back(total - end);
        view.pop_front(begin);
        out->append(std::move(view));
    }
};

class ResponseMerger {
public:
    enum Result { MERGED, FAIL, FAIL_ALL };
    virtual ~ResponseMerger() {}
    virtual Result Merge(pb::Message* response, const pb::Message* sub_response) = 0;
};

struct ParallelChannelOptions {
    int32_t timeout_ms = 500;   // -1: none
    int fail_limit = -1;        // finish as failed once this many sub calls failed (-1: all)
    int success_limit = -1;     // finish as ok once this many succeeded (-1: all)
    // MI355X extension (off by default, like the reference, whose parallel
    // channel only forwards the REQUEST attachment, parallel_channel.cpp:
    // 683-684): append the response attachments of the sub calls that
    // succeeded to the parent's response attachment, in channel order —
    // the gather half of a scatter/gather over device payloads (blocks are
    // shared, HBM blocks stay in HBM). With success_limit < n the gathered
    // set is the sub calls that had succeeded when the call finished.
    bool gather_response_attachments = false;
};

class ParallelChannel : public ChannelBase {
public:
    ParallelChannel() {}
    ~ParallelChannel() override;
    int Init(const ParallelChannelOptions* options);
    // mapper/merger may be null (request broadcast / MergeFrom). Shared
    // mappers and mergers are reference counted by the channel.
    int AddChannel(ChannelBase* sub, ChannelOwnership ownership, std::shared_ptr<CallMapper> mapper,
                   std::shared_ptr<ResponseMerger> merger);
    void Reset();
    int channel_count() const { return (int)_subs.size(); }
    void CallMethod(const pb::MethodDescriptor* method, RpcController* controller, const pb::Message* request,
                    pb::Message* response, Closure* done) override;
    int Weight() override;
    int CheckHealth() override;
    const ParallelChannelOptions& options() const { return _options; }

private:
    struct Sub {
        ChannelBase* channel;
        ChannelOwnership ownership;
        std::shared_ptr<CallMapper> mapper;
        std::shared_ptr<ResponseMerger> merger;
    };
    ParallelChannelOptions _options;
    std::vector<Sub> _subs;
};

// Parses a server tag into (index, total); "2/4" -> (2, 4) by default.
class PartitionParser {
public:
    virtual ~PartitionParser() {}
    struct Partition {
        int index = -1;
        int num_partition_kinds = 0;
    };
    virtual bool ParseFromTag(const std::string& tag, Partition* out);
};

struct PartitionChannelOptions : public ChannelOptions {
    int fail_limit = -1;
    int success_limit = -1;
    std::shared_ptr<CallMapper> call_mapper;
    std::shared_ptr<ResponseMerger> response_merger;
};

class PartitionChannel : public ChannelBase {
public:
    PartitionChannel() {}
    ~PartitionChannel() override;
    // Servers of `ns_url` tagged "i/num_partition_kinds" form partition i.
    int Init(int num_partition_kinds, PartitionParser* parser, const char* ns_url, const char* lb_name,
             const PartitionChannelOptions* options);
    int partition_count() const { return _num; }
    void CallMethod(const pb::MethodDescriptor* method, RpcController* controller, const pb::Message* request,
                    pb::Message* response, Closure* done) override;
    int Weight() override { return _pchan.Weight(); }
    int CheckHealth() override { return _pchan.CheckHealth(); }

private:
    int _num = 0;
    ParallelChannel _pchan;
    std::vector<std::unique_ptr<NamingServiceFilter>> _filters;
};

class DynamicPartitionChannel : public ChannelBase {
public:
    DynamicPartitionChannel();
    ~DynamicPartitionChannel() override;
    int Init(PartitionParser* parser, const char* ns_url, const char* lb_name, const PartitionChannelOptions* options);
    void CallMethod(const pb::MethodDescriptor* method, RpcController* controller, const pb::Message* request,
                    pb::Message* response, Closure* done) override;
    int Weight() override;
    int CheckHealth() override;
    // Number of partition schemes currently served (for tests/status).
    int scheme_count() const;
    // Re-resolve the naming service now (also done periodically).
    void Refresh();

private:
    struct Scheme;
    std::shared_ptr<Scheme> pick() const;
    static void* refresh_loop(void* arg);
    PartitionParser* _parser = nullptr;
    std::unique_ptr<PartitionParser> _default_parser;
    std::string _ns_url, _lb_name;
    PartitionChannelOptions _options;
    mutable std::mutex _mu;
    std::vector<std::shared_ptr<Scheme>> _schemes;
    std::atomic<bool> _stop{false};
    uint64_t _fiber = 0;
};

struct SelectiveChannelOptions {
    int32_t timeout_ms = 500;
    int32_t backup_request_ms = -1;
    int max_retry = 3;
    std::string lb = "rr";  // rr | random | wr (weighted by Weight()) | la (latency aware)
};

class SelectiveChannel : public ChannelBase {
public:
    SelectiveChannel() {}
    ~SelectiveChannel() override;
    int Init(const char* lb_name, const ChannelOptions* options);
    int Init(const SelectiveChannelOptions* options);
    // Returns a handle usable with RemoveAndDestroyChannel.
    int AddChannel(ChannelBase* sub, ChannelOwnership ownership = OWNS_CHANNEL, int weight = 1);
    void RemoveAndDestroyChannel(int handle);
    void CallMethod(const pb::MethodDescriptor* method, RpcController* controller, const pb::Message* request,
                    pb::Message* response, Closure* done) override;
    int Weight() override;
    int CheckHealth() override;

    struct Sub;
    struct Call;
    // index of the next sub channel to try (internal; used by calls)
    int select(const std::vector<int>& excluded);

private:
    friend struct Call;
    SelectiveChannelOptions _options;
    mutable std::mutex _mu;
    std::vector<std::shared_ptr<Sub>> _subs;
    std::atomic<uint64_t> _rr{0};
};

}  // namespace mrpc
