#include "var/reducer.h"

#include <vector>

namespace mrpc {
namespace var {
namespace detail {

namespace {
struct IdTable {
    std::vector<uint64_t> gens;  // current generation of each id; 0 = free
    std::vector<int> free_ids;
    uint64_t next_gen = 1;
};
IdTable& ids() {
    static IdTable* t = new IdTable;
    return *t;
}

struct TLSAgents {
    std::vector<AgentBase*> v;
    ~TLSAgents() {
        std::lock_guard<std::mutex> g(global_agent_mutex());
        for (AgentBase* a : v) {
            if (!a) continue;
            a->merge_and_detach();
            delete a;
        }
        v.clear();
    }
};
thread_local TLSAgents tls_agents;
}  // namespace

std::mutex& global_agent_mutex() {
    static std::mutex* m = new std::mutex;
    return *m;
}

void allocate_combiner_id(int* id, uint64_t* gen) {
    std::lock_guard<std::mutex> g(global_agent_mutex());
    IdTable& t = ids();
    int i;
    if (!t.free_ids.empty()) {
        i = t.free_ids.back();
        t.free_ids.pop_back();
    } else {
        i = (int)t.gens.size();
        t.gens.push_back(0);
    }
    t.gens[i] = t.next_gen++;
    *id = i;
    *gen = t.gens[i];
}

void free_combiner_id(int id) {
    // global lock held by caller
    IdTable& t = ids();
    t.gens[id] = 0;
    t.free_ids.push_back(id);
}

bool combiner_alive(int id, uint64_t gen) {
    IdTable& t = ids();
    return id >= 0 && id < (int)t.gens.size() && t.gens[id] == gen;
}

AgentBase* get_tls_agent(int id, uint64_t gen) {
    auto& v = tls_agents.v;
    if ((size_t)id < v.size()) {
        AgentBase* a = v[id];
        if (a && a->gen == gen) return a;
    }
    return nullptr;
}

void set_tls_agent(int id, AgentBase* a) {
    auto& v = tls_agents.v;
    if ((size_t)id >= v.size()) v.resize(id + 1, nullptr);
    AgentBase* old = v[id];
    v[id] = a;
    if (old) {
        // stale agent of a destroyed combiner that reused this id
        std::lock_guard<std::mutex> g(global_agent_mutex());
        old->merge_and_detach();
        delete old;
    }
}

}  // namespace detail
}  // namespace var
}  // namespace mrpc
