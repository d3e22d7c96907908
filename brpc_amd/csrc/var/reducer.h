// Reducers over thread-local agents (role of bvar/reducer.h:69,224,258,308
// and detail/combiner.h:156): writes touch only the calling thread's agent
// (an uncontended relaxed atomic, ~ns per update, flat in thread count);
// reads combine all agents. Adder/Maxer/Miner are the building blocks of
// windows, per-second rates and latency recorders.
#pragma once

#include <atomic>
#include <cstdint>
#include <limits>
#include <mutex>
#include <vector>

#include "var/variable.h"

namespace mrpc {
namespace var {
namespace detail {

struct AgentBase {
    virtual ~AgentBase() {}
    virtual void merge_and_detach() = 0;  // called at thread exit with global lock held
    uint64_t gen = 0;
};

std::mutex& global_agent_mutex();
// Allocates a (id, generation) pair for a combiner.
void allocate_combiner_id(int* id, uint64_t* gen);
void free_combiner_id(int id);
bool combiner_alive(int id, uint64_t gen);  // global lock must be held
// Thread-local agent table.
AgentBase* get_tls_agent(int id, uint64_t gen);
void set_tls_agent(int id, AgentBase* a);

template <typename T>
struct OpAdd {
    static T identity() { return T(0); }
    static T apply(T a, T b) { return a + b; }
    static void update(std::atomic<T>& a, T v) {
        if constexpr (std::is_integral<T>::value) {
            a.fetch_add(v, std::memory_order_relaxed);
        } else {
            // single writer per agent: load+store is enough
            a.store(a.load(std::memory_order_relaxed) + v, std::memory_order_relaxed);
        }
    }
    static bool inverse_ok() { return true; }
    static T inverse(T a, T b) { return a - b; }
};

template <typename T>
struct OpMax {
    static T identity() { return std::numeric_limits<T>::lowest(); }
    static T apply(T a, T b) { return a > b ? a : b; }
    static void update(std::atomic<T>& a, T v) {
        T cur = a.load(std::memory_order_relaxed);
        while (v > cur && !a.compare_exchange_weak(cur, v, std::memory_order_relaxed)) {
        }
    }
    static bool inverse_ok() { return false; }
    static T inverse(T a, T) { return a; }
};

template <typename T>
struct OpMin {
    static T identity() { return std::numeric_limits<T>::max(); }
    static T apply(T a, T b) { return a < b ? a : b; }
    static void update(std::atomic<T>& a, T v) {
        T cur = a.load(std::memory_order_relaxed);
        while (v < cur && !a.compare_exchange_weak(cur, v, std::memory_order_relaxed)) {
        }
    }
    static bool inverse_ok() { return false; }
    static T inverse(T a, T) { return a; }
};

template <typename T, typename Op>
class Combiner {
public:
    struct Agent : public AgentBase {
        std::atomic<T> value{Op::identity()};
        Combiner* owner = nullptr;
        void merge_and_detach() override {
            if (owner) owner->merge_global_and_remove(this);
            owner = nullptr;
        }
    };

    Combiner() : _global(Op::identity()) { allocate_combiner_id(&_id, &_gen); }
    ~Combiner() {
        std::lock_guard<std::mutex> g(global_agent_mutex());
        std::lock_guard<std::mutex> g2(_mu);
        for (Agent* a : _agents) a->owner = nullptr;
        _agents.clear();
        free_combiner_id(_id);
    }

    Agent* agent() {
        AgentBase* a = get_tls_agent(_id, _gen);
        if (__builtin_expect(a != nullptr, 1)) return static_cast<Agent*>(a);
        Agent* na = new Agent;
        na->gen = _gen;
        na->owner = this;
        {
            std::lock_guard<std::mutex> g(_mu);
            _agents.push_back(na);
        }
        set_tls_agent(_id, na);
        return na;
    }

    T combine() const {
        std::lock_guard<std::mutex> g(_mu);
        T r = _global;
        for (Agent* a : _agents) r = Op::apply(r, a->value.load(std::memory_order_relaxed));
        return r;
    }

    // For Maxer/Miner windows: return combined value and reset all agents.
    T reset() {
        std::lock_guard<std::mutex> g(_mu);
        T r = _global;
        _global = Op::identity();
        for (Agent* a : _agents) r = Op::apply(r, a->value.exchange(Op::identity(), std::memory_order_relaxed));
        return r;
    }

    void merge_global_and_remove(Agent* a) {
        std::lock_guard<std::mutex> g(_mu);
        _global = Op::apply(_global, a->value.load(std::memory_order_relaxed));
        for (size_t i = 0; i < _agents.size(); ++i) {
            if (_agents[i] == a) {
                _agents[i] = _agents.back();
                _agents.pop_back();
                break;
            }
        }
    }

private:
    int _id;
    uint64_t _gen;
    mutable std::mutex _mu;
    T _global;
    std::vector<Agent*> _agents;
};

}  // namespace detail

template <typename T, typename Op>
class Reducer : public Variable {
public:
    typedef T value_type;
    typedef Op op_type;
    Reducer() {}
    Reducer& operator<<(T v) {
        Op::update(_combiner.agent()->value, v);
        return *this;
    }
    T get_value() const { return _combiner.combine(); }
    T reset() { return _combiner.reset(); }
    void describe(std::ostream& os, bool) const override { os << get_value(); }
    bool get_number(double* out) const override {
        *out = (double)get_value();
        return true;
    }

private:
    mutable detail::Combiner<T, Op> _combiner;
};

template <typename T = int64_t>
class Adder : public Reducer<T, detail::OpAdd<T>> {
public:
    Adder() {}
    explicit Adder(const std::string& name) { this->expose(name); }
    Adder(const std::string& prefix, const std::string& name) { this->expose_as(prefix, name); }
};

template <typename T = int64_t>
class Maxer : public Reducer<T, detail::OpMax<T>> {
public:
    Maxer() {}
    explicit Maxer(const std::string& name) { this->expose(name); }
    Maxer(const std::string& prefix, const std::string& name) { this->expose_as(prefix, name); }
    void describe(std::ostream& os, bool) const override {
        T v = this->get_value();
        os << (v == detail::OpMax<T>::identity() ? T(0) : v);
    }
};

template <typename T = int64_t>
class Miner : public Reducer<T, detail::OpMin<T>> {
public:
    Miner() {}
    explicit Miner(const std::string& name) { this->expose(name); }
    void describe(std::ostream& os, bool) const override {
        T v = this->get_value();
        os << (v == detail::OpMin<T>::identity() ? T(0) : v);
    }
};

}  // namespace var
}  // namespace mrpc
