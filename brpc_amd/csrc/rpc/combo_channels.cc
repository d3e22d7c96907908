#include "rpc/combo_channels.h"

#include <algorithm>
#include <cmath>
#include <fstream>
#include <map>

#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/call_id.h"
#include "fiber/fiber.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/retry_policy.h"

namespace mrpc {

// =================================================================== Parallel
namespace {

struct PCall;

struct SubState {
    PCall* pc = nullptr;
    int index = 0;
    SubCall sc;
    Controller cntl;
    bool launched = false;
    bool succeeded = false;  // set under PCall::mu
};

struct PCall {
    Controller* cntl = nullptr;
    pb::Message* response = nullptr;
    Closure* done = nullptr;
    fiber::CallId cid{0};
    std::vector<std::unique_ptr<SubState>> subs;
    std::vector<std::shared_ptr<ResponseMerger>> mergers;
    std::mutex mu;
    int nlaunched = 0, nfail = 0, nsuccess = 0, ndone = 0;
    int fail_limit = 0, success_limit = 0;
    bool gather = false;  // ParallelChannelOptions::gather_response_attachments
    bool finished = false;
    bool canceled = false;  // the parent was canceled
    int first_error = 0;
    int unified_error = 0;  // the failed sub calls' common code (ECANCELED aside), or ETOOMANYFAILS
    std::string first_error_text;
    std::atomic<int> refs{1};

    void unref() {
        if (refs.fetch_sub(1) == 1) delete this;
    }
    ~PCall() {
        for (auto& s : subs) {
            if (s->sc.flags & SubCall::DELETE_REQUEST) delete s->sc.request;
            if (s->sc.flags & SubCall::DELETE_RESPONSE) delete s->sc.response;
        }
    }
};

// Completes the parent RPC (exactly once).
void finish_parent(PCall* pc, int error_code, const std::string& text) {
    Controller* cntl = pc->cntl;
    if (error_code) cntl->SetFailed(error_code, "%s", text.c_str());
    // opt-in gather: the response attachments of the sub calls that
    // succeeded, in channel order (blocks are shared, HBM blocks stay in HBM)
    if (!error_code && pc->gather) {
        std::lock_guard<std::mutex> g(pc->mu);
        for (auto& s : pc->subs) {
            if (s->succeeded) cntl->response_attachment().append(s->cntl.response_attachment());
        }
    }
    cntl->_end_us = monotonic_us();
    Closure* done = pc->done;
    const fiber::CallId cid = pc->cid;
    cntl->_ended_id = cid;
    __atomic_store_n(&cntl->_correlation_id.value, 0, __ATOMIC_RELEASE);  // pairs with Controller::Join
    // cancel sub calls still in flight; their done closures only unref
    for (auto& s : pc->subs) {
        if (s->launched) s->cntl.StartCancel();
    }
    if (fiber::call_id_lock(cid, nullptr) == 0) fiber::call_id_unlock_and_destroy(cid);
    if (done) done->Run();
}

void on_sub_done(SubState* s) {
    PCall* pc = s->pc;
    bool complete = false;
    int ec = 0;
    std::string et;
    {
        std::lock_guard<std::mutex> g(pc->mu);
        ++pc->ndone;
        if (!pc->finished) {
            bool ok = !s->cntl.Failed();
            if (ok && s->sc.response && pc->response) {
                ResponseMerger* m = pc->mergers[s->index].get();
                if (m) {
                    const ResponseMerger::Result r = m->Merge(pc->response, s->sc.response);
                    if (r == ResponseMerger::FAIL) {
                        ok = false;
                        s->cntl.SetFailed(ERESPONSE, "merger failed sub call %d", s->index);
                    } else if (r == ResponseMerger::FAIL_ALL) {
                        pc->finished = true;
                        complete = true;
                        ec = ERESPONSE;
                        et = "merger asked to fail all (sub call " + std::to_string(s->index) + ")";
                    }
                } else if (s->sc.response != pc->response) {
                    pc->response->MergeFrom(*s->sc.response);
                }
            }
            if (!pc->finished) {
                if (ok) {
                    s->succeeded = true;
                    ++pc->nsuccess;
                } else {
                    ++pc->nfail;
                    const int sec = s->cntl.ErrorCode();
                    if (!pc->first_error) {
                        pc->first_error = sec;
                        pc->first_error_text = s->cntl.ErrorText();
                    }
                    if (sec != ECANCELED) {
                        if (pc->unified_error == 0) pc->unified_error = sec;
                        else if (pc->unified_error != sec) pc->unified_error = ETOOMANYFAILS;
                    }
                }
                if (pc->nfail >= pc->fail_limit) {
                    pc->finished = true;
                    complete = true;
                    // the reference's unified code (parallel_channel.cpp:352-366):
                    // the failed sub calls' common error, ECANCELED when they
                    // were all canceled, ETOOMANYFAILS when they differ
                    ec = pc->unified_error ? pc->unified_error : ECANCELED;
                    et = std::to_string(pc->nfail) + "/" + std::to_string(pc->nlaunched) +
                         " sub calls failed (fail_limit=" + std::to_string(pc->fail_limit) +
                         "), first: [E" + std::to_string(pc->first_error) + "] " + pc->first_error_text;
                } else if (pc->nsuccess >= pc->success_limit || pc->ndone == pc->nlaunched) {
                    // (a canceled call whose failures stayed under fail_limit
                    // succeeds: enough sub calls succeeded before the cancel,
                    // parallel_channel.cpp:375-381)
                    pc->finished = true;
                    complete = true;
                }
            }
        }
    }
    if (complete) finish_parent(pc, ec, et);
    pc->unref();
}

int OnParallelError(fiber::CallId id, void* data, int error_code, const std::string& text) {
    PCall* pc = static_cast<PCall*>(data);
    // cancellation / timeout of the parent: cancel the sub calls and let
    // them complete the parent through the fail path. The id is released
    // first: a canceled sub call may complete inline, and the last one
    // finishes the parent, which locks this id.
    pc->refs.fetch_add(1);
    if (error_code == ECANCELED) {
        std::lock_guard<std::mutex> g(pc->mu);
        pc->canceled = true;
    }
    fiber::call_id_unlock(id);
    for (auto& s : pc->subs) {
        if (s->launched) s->cntl.StartCancel();
    }
    pc->unref();
    (void)error_code;
    (void)text;
    return 0;
}

// A controller canceled before CallMethod (StartCancel on its call_id()):
// the combo call ends at once with ECANCELED and issues no sub call, like a
// plain Channel's.
bool canceled_before_call(Controller* cntl, Closure* done) {
    if (!cntl->Failed() || cntl->ErrorCode() != ECANCELED) return false;
    if (done) done->Run();
    return true;
}

}  // namespace

ParallelChannel::~ParallelChannel() { Reset(); }

int ParallelChannel::Init(const ParallelChannelOptions* options) {
    if (options) _options = *options;
    return 0;
}

int ParallelChannel::AddChannel(ChannelBase* sub, ChannelOwnership ownership, std::shared_ptr<CallMapper> mapper,
                                std::shared_ptr<ResponseMerger> merger) {
    if (!sub) return -1;
    _subs.push_back(Sub{sub, ownership, std::move(mapper), std::move(merger)});
    return 0;
}

void ParallelChannel::Reset() {
    for (Sub& s : _subs) {
        if (s.ownership == OWNS_CHANNEL) delete s.channel;
    }
    _subs.clear();
}

int ParallelChannel::Weight() {
    int w = 0;
    for (Sub& s : _subs) w += s.channel->Weight();
    return w;
}

int ParallelChannel::CheckHealth() {
    if (_subs.empty()) return -1;
    int healthy = 0;
    for (Sub& s : _subs) healthy += s.channel->CheckHealth() == 0;
    const int need = _options.fail_limit < 0 ? 1 : std::max(1, (int)_subs.size() - _options.fail_limit + 1);
    return healthy >= need ? 0 : -1;
}

void ParallelChannel::CallMethod(const pb::MethodDescriptor* method, RpcController* controller_base,
                                 const pb::Message* request, pb::Message* response, Closure* done) {
    Controller* cntl = static_cast<Controller*>(controller_base);
    cntl->_begin_us = monotonic_us();
    if (canceled_before_call(cntl, done)) return;
    const int n = (int)_subs.size();
    PCall* pc = new PCall;
    pc->cntl = cntl;
    pc->response = response;
    pc->done = done;
    if (fiber::call_id_create(&pc->cid, pc, OnParallelError) != 0) {
        delete pc;
        cntl->SetFailed(EINTERNAL, "fail to create call id");
        if (done) done->Run();
        return;
    }
    fiber::call_id_lock(pc->cid, nullptr);
    cntl->_correlation_id = pc->cid;
    const int64_t timeout_ms = cntl->timeout_ms() != Controller::UNSET_MAGIC ? cntl->timeout_ms()
                                                                               : _options.timeout_ms;
    int nbad = 0;
    for (int i = 0; i < n; ++i) {
        std::unique_ptr<SubState> s(new SubState);
        s->pc = pc;
        s->index = i;
        if (_subs[i].mapper) {
            s->sc = _subs[i].mapper->Map(i, n, method, request, response);
        } else {
            s->sc = SubCall(method, request, response ? response->New() : nullptr, SubCall::DELETE_RESPONSE);
        }
        if (s->sc.is_bad()) ++nbad;
        pc->mergers.push_back(_subs[i].merger);
        pc->subs.push_back(std::move(s));
    }
    // finish_parent locks the call id itself: release ours first (the
    // early exits below used to self-deadlock on it)
    if (nbad) {
        fiber::call_id_unlock(pc->cid);
        finish_parent(pc, EREQUEST, "CallMapper returned Bad() for " + std::to_string(nbad) + " sub calls");
        pc->unref();
        return;
    }
    for (auto& s : pc->subs) {
        if (!s->sc.is_skip()) ++pc->nlaunched;
    }
    if (pc->nlaunched == 0) {
        fiber::call_id_unlock(pc->cid);
        finish_parent(pc, EREQUEST, "all sub calls are skipped");
        pc->unref();
        return;
    }
    pc->fail_limit = _options.fail_limit < 0 ? pc->nlaunched : std::max(1, _options.fail_limit);
    pc->success_limit = _options.success_limit < 0 ? pc->nlaunched : std::max(1, _options.success_limit);
    pc->gather = _options.gather_response_attachments;
    pc->refs.fetch_add(pc->nlaunched);
    std::vector<SubState*> to_launch;
    for (auto& s : pc->subs) {
        if (s->sc.is_skip()) continue;
        s->launched = true;
        s->cntl.set_timeout_ms(timeout_ms);
        if (cntl->log_id()) s->cntl.set_log_id(cntl->log_id());
        if (cntl->has_request_code()) s->cntl.set_request_code(cntl->request_code());
        // every sub call carries the attachment, or the mapper's slice of it
        // (shared blocks, no copy; reference parallel_channel.cpp:683-684)
        if (_subs[s->index].mapper) {
            _subs[s->index].mapper->MapAttachment(s->index, (int)_subs.size(), cntl->request_attachment(),
                                                  &s->cntl.request_attachment());
        } else {
            s->cntl.request_attachment().append(cntl->request_attachment());
        }
        to_launch.push_back(s.get());
    }
    const fiber::CallId cid = pc->cid;
    fiber::call_id_unlock(cid);  // sub calls may finish the parent from now on
    for (SubState* s : to_launch) {
        _subs[s->index].channel->CallMethod(s->sc.method, &s->cntl, s->sc.request, s->sc.response,
                                            NewCallback([s] { on_sub_done(s); }));
    }
    pc->unref();
    if (!done) fiber::call_id_join(cid);
}

// =================================================================== Partition
bool PartitionParser::ParseFromTag(const std::string& tag, Partition* out) {
    const size_t slash = tag.find('/');
    if (slash == std::string::npos) return false;
    char* e1 = nullptr;
    char* e2 = nullptr;
    const long idx = strtol(tag.c_str(), &e1, 10);
    const long num = strtol(tag.c_str() + slash + 1, &e2, 10);
    if (e1 != tag.c_str() + slash || num <= 0 || idx < 0 || idx >= num) return false;
    out->index = (int)idx;
    out->num_partition_kinds = (int)num;
    return true;
}

namespace {
class PartitionFilter : public NamingServiceFilter {
public:
    PartitionFilter(PartitionParser* p, int index, int num) : _p(p), _index(index), _num(num) {}
    bool Accept(const ServerNode& s) const override {
        PartitionParser::Partition part;
        return _p->ParseFromTag(s.tag, &part) && part.index == _index && part.num_partition_kinds == _num;
    }

private:
    PartitionParser* _p;
    int _index, _num;
};
}  // namespace

PartitionChannel::~PartitionChannel() { _pchan.Reset(); }

int PartitionChannel::Init(int num_partition_kinds, PartitionParser* parser, const char* ns_url,
                           const char* lb_name, const PartitionChannelOptions* options) {
    if (num_partition_kinds <= 0 || !parser) return -1;
    PartitionChannelOptions opt = options ? *options : PartitionChannelOptions();
    ParallelChannelOptions popt;
    popt.timeout_ms = opt.timeout_ms;
    popt.fail_limit = opt.fail_limit;
    popt.success_limit = opt.success_limit;
    _pchan.Init(&popt);
    _num = num_partition_kinds;
    for (int i = 0; i < num_partition_kinds; ++i) {
        _filters.emplace_back(new PartitionFilter(parser, i, num_partition_kinds));
        ChannelOptions co = opt;
        co.ns_filter = _filters.back().get();
        co.succeed_without_server = true;
        Channel* ch = new Channel;
        if (ch->Init(ns_url, lb_name, &co) != 0) {
            delete ch;
            LOG(ERROR) << "Fail to init partition " << i << " of " << ns_url;
            return -1;
        }
        _pchan.AddChannel(ch, OWNS_CHANNEL, opt.call_mapper, opt.response_merger);
    }
    return 0;
}

void PartitionChannel::CallMethod(const pb::MethodDescriptor* method, RpcController* controller,
                                  const pb::Message* request, pb::Message* response, Closure* done) {
    _pchan.CallMethod(method, controller, request, response, done);
}

// ============================================================ DynamicPartition
struct DynamicPartitionChannel::Scheme {
    int num = 0;
    int nservers = 0;
    std::string signature;  // sorted server list, to skip unchanged rebuilds
    std::unique_ptr<PartitionChannel> channel;
};

DynamicPartitionChannel::DynamicPartitionChannel() {}

DynamicPartitionChannel::~DynamicPartitionChannel() {
    _stop.store(true);
    if (_fiber) {
        fiber::stop(_fiber);
        fiber::join(_fiber);
    }
}

int DynamicPartitionChannel::Init(PartitionParser* parser, const char* ns_url, const char* lb_name,
                                  const PartitionChannelOptions* options) {
    if (!parser) {
        _default_parser.reset(new PartitionParser);
        parser = _default_parser.get();
    }
    _parser = parser;
    _ns_url = ns_url;
    _lb_name = lb_name ? lb_name : "rr";
    if (options) _options = *options;
    Refresh();
    fiber::Attr attr(fiber::STACK_NORMAL, fiber::ATTR_NOSIGNAL);
    fiber::fiber_t tid;
    if (fiber::start_background(&tid, &attr, refresh_loop, this) == 0) _fiber = tid;
    return 0;
}

void* DynamicPartitionChannel::refresh_loop(void* arg) {
    DynamicPartitionChannel* self = static_cast<DynamicPartitionChannel*>(arg);
    while (!self->_stop.load()) {
        if (fiber::usleep(1000000) != 0 && self->_stop.load()) break;
        if (!self->_stop.load()) self->Refresh();
    }
    return nullptr;
}

void DynamicPartitionChannel::Refresh() {
    const size_t pos = _ns_url.find("://");
    if (pos == std::string::npos) return;
    const std::string scheme = _ns_url.substr(0, pos);
    const std::string name = _ns_url.substr(pos + 3);
    std::vector<ServerNode> servers;
    if (scheme == "file") {
        // re-read the list every refresh (the file NS itself blocks forever)
        std::ifstream in(name);
        if (!in) return;
        std::string line;
        while (std::getline(in, line)) {
            ServerNode n;
            const std::string t = trim(line);
            if (!t.empty() && t[0] != '#' && ParseServerNode(t, &n)) servers.push_back(n);
        }
    } else {
        std::unique_ptr<NamingService> ns(CreateNamingService(scheme));
        if (!ns) return;
        if (PeriodicNamingService* pns = dynamic_cast<PeriodicNamingService*>(ns.get())) {
            if (pns->GetServers(name.c_str(), &servers) != 0) return;
        } else if (ns->RunNamingServiceReturnsQuickly()) {
            struct Collect : public NamingServiceActions {
                std::vector<ServerNode>* out;
                void ResetServers(const std::vector<ServerNode>& s) override { *out = s; }
            } c;
            c.out = &servers;
            if (ns->RunNamingService(name.c_str(), &c) != 0) return;
        } else {
            return;
        }
    }
    std::map<int, std::vector<ServerNode>> by_num;
    for (const ServerNode& s : servers) {
        PartitionParser::Partition p;
        if (_parser->ParseFromTag(s.tag, &p)) by_num[p.num_partition_kinds].push_back(s);
    }
    std::vector<std::shared_ptr<Scheme>> next;
    std::vector<std::shared_ptr<Scheme>> old;
    {
        std::lock_guard<std::mutex> g(_mu);
        old = _schemes;
    }
    for (auto& kv : by_num) {
        std::vector<ServerNode>& list = kv.second;
        std::sort(list.begin(), list.end());
        std::string sig;
        for (const ServerNode& s : list) sig += s.addr.to_string() + " " + s.tag + ",";
        std::shared_ptr<Scheme> reuse;
        for (auto& o : old) {
            if (o->num == kv.first && o->signature == sig) reuse = o;
        }
        if (reuse) {
            next.push_back(reuse);
            continue;
        }
        auto sc = std::make_shared<Scheme>();
        sc->num = kv.first;
        sc->nservers = (int)list.size();
        sc->signature = sig;
        sc->channel.reset(new PartitionChannel);
        std::string url = "list://";
        for (size_t i = 0; i < list.size(); ++i) {
            url += (i ? "," : "") + list[i].addr.to_string() + " " + list[i].tag;
        }
        if (sc->channel->Init(kv.first, _parser, url.c_str(), _lb_name.c_str(), &_options) != 0) continue;
        next.push_back(sc);
    }
    std::lock_guard<std::mutex> g(_mu);
    _schemes.swap(next);
}

std::shared_ptr<DynamicPartitionChannel::Scheme> DynamicPartitionChannel::pick() const {
    std::lock_guard<std::mutex> g(_mu);
    if (_schemes.empty()) return nullptr;
    // capacity of a scheme = servers per partition; split traffic by it
    int64_t total = 0;
    for (auto& s : _schemes) total += std::max(1, s->nservers / std::max(1, s->num));
    int64_t r = (int64_t)(fast_rand() % (uint64_t)total);
    for (auto& s : _schemes) {
        r -= std::max(1, s->nservers / std::max(1, s->num));
        if (r < 0) return s;
    }
    return _schemes.back();
}

int DynamicPartitionChannel::scheme_count() const {
    std::lock_guard<std::mutex> g(_mu);
    return (int)_schemes.size();
}

void DynamicPartitionChannel::CallMethod(const pb::MethodDescriptor* method, RpcController* controller,
                                         const pb::Message* request, pb::Message* response, Closure* done) {
    std::shared_ptr<Scheme> s = pick();
    if (!s) {
        Controller* cntl = static_cast<Controller*>(controller);
        cntl->SetFailed(EHOSTDOWN, "no partition scheme available from %s", _ns_url.c_str());
        if (done) done->Run();
        return;
    }
    // keep the scheme alive until the call ends
    if (done) {
        Closure* inner = done;
        done = NewCallback([s, inner] { inner->Run(); });
    }
    s->channel->CallMethod(method, controller, request, response, done);
}

int DynamicPartitionChannel::Weight() {
    std::lock_guard<std::mutex> g(_mu);
    int w = 0;
    for (auto& s : _schemes) w += s->channel->Weight();
    return w;
}

int DynamicPartitionChannel::CheckHealth() { return scheme_count() > 0 ? 0 : -1; }

// =================================================================== Selective
struct SelectiveChannel::Sub {
    ChannelBase* channel;
    ChannelOwnership ownership;
    int weight;
    std::atomic<int64_t> ema_latency_us{0};
    std::atomic<int> inflight{0};
    std::atomic<int64_t> failures{0};
    bool removed = false;
    ~Sub() {
        if (ownership == OWNS_CHANNEL) delete channel;
    }
};

struct SelectiveChannel::Call {
    SelectiveChannel* ch;
    Controller* cntl;
    const pb::MethodDescriptor* method;
    const pb::Message* request;
    pb::Message* response;
    Closure* done;
    fiber::CallId cid{0};
    std::mutex mu;
    std::vector<int> tried;
    int attempts = 0;
    bool finished = false;
    int inflight = 0;
    fiber::TimerId backup_timer = 0;
    bool backup_cancelled = false;
    bool canceled = false;            // under mu: the parent was canceled
    std::vector<Controller*> live;    // under mu: attempts in flight
    std::atomic<int> refs{1};
    void unref() {
        if (refs.fetch_sub(1) == 1) delete this;
    }

    struct Attempt {
        Call* call;
        std::shared_ptr<Sub> sub;
        int index;
        Controller sub_cntl;
        pb::Message* res;
        int64_t begin_us;
    };

    Attempt* prepare(int idx);
    void issue(Attempt* a);
    void on_attempt_done(Attempt* a);
    void finish(int ec, const std::string& text, pb::Message* res);
};

SelectiveChannel::~SelectiveChannel() {}

int SelectiveChannel::Init(const char* lb_name, const ChannelOptions* options) {
    if (lb_name) _options.lb = lb_name;
    if (options) {
        _options.timeout_ms = options->timeout_ms;
        _options.backup_request_ms = options->backup_request_ms;
        _options.max_retry = options->max_retry;
    }
    return 0;
}

int SelectiveChannel::Init(const SelectiveChannelOptions* options) {
    if (options) _options = *options;
    return 0;
}

int SelectiveChannel::AddChannel(ChannelBase* sub, ChannelOwnership ownership, int weight) {
    auto s = std::make_shared<Sub>();
    s->channel = sub;
    s->ownership = ownership;
    s->weight = std::max(1, weight);
    std::lock_guard<std::mutex> g(_mu);
    _subs.push_back(s);
    return (int)_subs.size() - 1;
}

void SelectiveChannel::RemoveAndDestroyChannel(int handle) {
    std::lock_guard<std::mutex> g(_mu);
    if (handle < 0 || handle >= (int)_subs.size() || !_subs[handle]) return;
    _subs[handle]->removed = true;
    _subs[handle].reset();  // destroyed when the last in-flight attempt ends
}

int SelectiveChannel::Weight() {
    std::lock_guard<std::mutex> g(_mu);
    int w = 0;
    for (auto& s : _subs) w += s ? s->weight : 0;
    return w;
}

int SelectiveChannel::CheckHealth() {
    std::lock_guard<std::mutex> g(_mu);
    for (auto& s : _subs) {
        if (s && s->channel->CheckHealth() == 0) return 0;
    }
    return -1;
}

int SelectiveChannel::select(const std::vector<int>& excluded) {
    std::lock_guard<std::mutex> g(_mu);
    std::vector<int> cand;
    for (int i = 0; i < (int)_subs.size(); ++i) {
        if (!_subs[i] || std::find(excluded.begin(), excluded.end(), i) != excluded.end()) continue;
        cand.push_back(i);
    }
    if (cand.empty()) {
        // everything tried: allow repeats of healthy ones
        for (int i = 0; i < (int)_subs.size(); ++i) {
            if (_subs[i]) cand.push_back(i);
        }
        if (cand.empty()) return -1;
    }
    if (_options.lb == "random") return cand[fast_rand() % cand.size()];
    if (_options.lb == "wr" || _options.lb == "wrr") {
        int64_t total = 0;
        for (int i : cand) total += _subs[i]->weight;
        int64_t r = (int64_t)(fast_rand() % (uint64_t)total);
        for (int i : cand) {
            r -= _subs[i]->weight;
            if (r < 0) return i;
        }
        return cand.back();
    }
    if (_options.lb == "la") {
        // smallest expected latency x (inflight+1), ties broken randomly
        int best = -1;
        double best_cost = 0;
        for (int i : cand) {
            const double lat = (double)std::max<int64_t>(1, _subs[i]->ema_latency_us.load());
            const double cost = lat * (_subs[i]->inflight.load() + 1) / _subs[i]->weight;
            if (best < 0 || cost < best_cost) {
                best = i;
                best_cost = cost;
            }
        }
        return best;
    }
    return cand[_rr.fetch_add(1) % cand.size()];
}

void SelectiveChannel::Call::finish(int ec, const std::string& text, pb::Message* res) {
    // called with mu held, finished == false
    finished = true;
    if (backup_timer && fiber::timer_del(backup_timer) == 0) backup_cancelled = true;  // timer's ref is ours now
    backup_timer = 0;
    if (ec) cntl->SetFailed(ec, "%s", text.c_str());
    else if (res && response && res != response) response->CopyFrom(*res);
    cntl->_end_us = monotonic_us();
}

// Bookkeeping of a new attempt; called with `mu` held. The sub call itself
// is issued by issue() after `mu` is released (its done may run inline).
SelectiveChannel::Call::Attempt* SelectiveChannel::Call::prepare(int idx) {
    std::shared_ptr<Sub> sub;
    {
        std::lock_guard<std::mutex> g(ch->_mu);
        if (idx >= 0 && idx < (int)ch->_subs.size()) sub = ch->_subs[idx];
    }
    if (!sub) return nullptr;
    Attempt* a = new Attempt;
    a->call = this;
    a->sub = sub;
    a->index = idx;
    a->res = response ? response->New() : nullptr;
    a->begin_us = monotonic_us();
    const int64_t remain_ms = cntl->timeout_ms() > 0 ? std::max<int64_t>(
                                                           1, cntl->timeout_ms() - (monotonic_us() - cntl->_begin_us) / 1000)
                                                     : -1;
    a->sub_cntl.set_timeout_ms(remain_ms);
    a->sub_cntl.set_max_retry(0);
    if (cntl->log_id()) a->sub_cntl.set_log_id(cntl->log_id());
    if (cntl->has_request_code()) a->sub_cntl.set_request_code(cntl->request_code());
    a->sub_cntl.request_attachment() = cntl->request_attachment();
    sub->inflight.fetch_add(1);
    refs.fetch_add(1);
    ++inflight;
    ++attempts;
    tried.push_back(idx);
    a->sub_cntl.call_id();  // created now, so a cancel between here and issue() reaches it
    live.push_back(&a->sub_cntl);
    return a;
}

void SelectiveChannel::Call::issue(Attempt* a) {
    if (!a) return;
    a->sub->channel->CallMethod(method, &a->sub_cntl, request, a->res,
                                NewCallback([a] { a->call->on_attempt_done(a); }));
}

void SelectiveChannel::Call::on_attempt_done(Attempt* a) {
    std::unique_ptr<Attempt> guard(a);
    std::unique_ptr<pb::Message> res(a->res);
    a->sub->inflight.fetch_sub(1);
    const int64_t lat = monotonic_us() - a->begin_us;
    if (!a->sub_cntl.Failed()) {
        const int64_t old = a->sub->ema_latency_us.load();
        a->sub->ema_latency_us.store(old ? (old * 7 + lat) / 8 : lat);
    } else {
        a->sub->failures.fetch_add(1);
    }
    bool complete = false;
    bool retry = false;
    {
        std::lock_guard<std::mutex> g(mu);
        --inflight;
        live.erase(std::remove(live.begin(), live.end(), &a->sub_cntl), live.end());
        if (!finished && canceled) {
            if (inflight == 0) {  // the parent was canceled: no retry, no late success
                finish(ECANCELED, "RPC canceled", nullptr);
                complete = true;
            }
        } else if (!finished) {
            if (!a->sub_cntl.Failed()) {
                cntl->response_attachment() = a->sub_cntl.response_attachment();
                finish(0, "", res.get());
                complete = true;
            } else if (a->sub_cntl.ErrorCode() != ERPCTIMEDOUT && a->sub_cntl.ErrorCode() != ECANCELED &&
                       DefaultRetryPolicy()->DoRetry(&a->sub_cntl) && attempts <= ch->_options.max_retry) {
                retry = true;
            } else if (inflight == 0) {
                finish(a->sub_cntl.ErrorCode(), a->sub_cntl.ErrorText(), nullptr);
                complete = true;
            }
        }
    }
    if (retry) {
        std::vector<int> excluded;
        {
            std::lock_guard<std::mutex> g(mu);
            excluded = tried;
        }
        const int idx = ch->select(excluded);
        Attempt* next = nullptr;
        {
            std::lock_guard<std::mutex> g(mu);
            if (!finished) {
                if (idx >= 0) {
                    next = prepare(idx);
                } else if (inflight == 0) {
                    finish(a->sub_cntl.ErrorCode(), a->sub_cntl.ErrorText(), nullptr);
                    complete = true;
                }
            }
        }
        issue(next);
    }
    if (complete) {
        Closure* d = done;
        const fiber::CallId id = cid;
        const bool drop_timer_ref = backup_cancelled;
        cntl->_ended_id = id;
        __atomic_store_n(&cntl->_correlation_id.value, 0, __ATOMIC_RELEASE);  // pairs with Controller::Join
        if (fiber::call_id_lock(id, nullptr) == 0) fiber::call_id_unlock_and_destroy(id);
        if (d) d->Run();
        if (drop_timer_ref) unref();
    }
    unref();
}

static void selective_backup(void* arg) {
    SelectiveChannel::Call* c = static_cast<SelectiveChannel::Call*>(arg);
    fiber::start([c] {
        std::vector<int> excluded;
        {
            std::lock_guard<std::mutex> g(c->mu);
            excluded = c->tried;
        }
        const int idx = c->ch->select(excluded);
        SelectiveChannel::Call::Attempt* a = nullptr;
        {
            std::lock_guard<std::mutex> g(c->mu);
            c->backup_timer = 0;
            if (!c->finished && idx >= 0) a = c->prepare(idx);
        }
        c->issue(a);
        c->unref();
    });
}

static int OnSelectiveError(fiber::CallId id, void* data, int error_code, const std::string&) {
    SelectiveChannel::Call* c = static_cast<SelectiveChannel::Call*>(data);
    if (error_code != ECANCELED) return fiber::call_id_unlock(id);  // attempts carry their own timeouts
    // canceled: cancel the attempts in flight; the last one to return
    // finishes the call with ECANCELED (the id is released first, an
    // attempt may complete inline)
    // an attempt may end (and free its controller) as soon as `mu` is
    // released: take the ids of the calls in flight, not the controllers,
    // and cancel by id (a stale id is a no-op)
    std::vector<fiber::CallId> live;
    c->refs.fetch_add(1);
    {
        std::lock_guard<std::mutex> g(c->mu);
        c->canceled = true;
        for (Controller* sc : c->live) live.push_back(sc->inflight_call_id());
    }
    fiber::call_id_unlock(id);
    for (fiber::CallId sid : live) {
        if (sid.value) StartCancel(sid);
    }
    c->unref();
    return 0;
}

void SelectiveChannel::CallMethod(const pb::MethodDescriptor* method, RpcController* controller,
                                  const pb::Message* request, pb::Message* response, Closure* done) {
    Controller* cntl = static_cast<Controller*>(controller);
    cntl->_begin_us = monotonic_us();
    if (canceled_before_call(cntl, done)) return;
    if (cntl->timeout_ms() == Controller::UNSET_MAGIC) cntl->set_timeout_ms(_options.timeout_ms);
    Call* c = new Call{this, cntl, method, request, response, done};
    fiber::call_id_create(&c->cid, c, OnSelectiveError);
    fiber::call_id_lock(c->cid, nullptr);
    cntl->_correlation_id = c->cid;
    const fiber::CallId cid = c->cid;
    const int idx = select({});
    if (idx < 0) {
        cntl->SetFailed(EHOSTDOWN, "SelectiveChannel has no sub channel");
        __atomic_store_n(&cntl->_correlation_id.value, 0, __ATOMIC_RELEASE);  // pairs with Controller::Join
        fiber::call_id_unlock_and_destroy(cid);
        c->unref();
        if (done) done->Run();
        return;
    }
    Call::Attempt* first = nullptr;
    {
        std::lock_guard<std::mutex> g(c->mu);
        first = c->prepare(idx);
        if (_options.backup_request_ms >= 0 && !c->finished) {
            c->refs.fetch_add(1);
            if (fiber::timer_add_us(&c->backup_timer, _options.backup_request_ms * 1000, selective_backup, c) != 0) {
                c->refs.fetch_sub(1);
                c->backup_timer = 0;
            }
        }
    }
    fiber::call_id_unlock(cid);  // the attempt's done may complete the call inline
    c->issue(first);
    c->unref();
    if (!done) fiber::call_id_join(cid);
}

}  // namespace mrpc
