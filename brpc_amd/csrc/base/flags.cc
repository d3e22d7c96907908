#include "base/flags.h"

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>

#include "base/logging.h"

namespace mrpc {

namespace {
struct FlagCell {
    std::string name;
    FlagType type;
    std::string desc;
    std::string file;
    void* storage;
    std::string default_value;
    FlagValidator validator;
    bool reloadable = false;
};

struct Registry {
    std::mutex mu;
    std::map<std::string, FlagCell> flags;
};

Registry& registry() {
    static Registry* r = new Registry;
    return *r;
}

const char* type_name(FlagType t) {
    switch (t) {
    case FlagType::BOOL: return "bool";
    case FlagType::INT32: return "int32";
    case FlagType::INT64: return "int64";
    case FlagType::UINT64: return "uint64";
    case FlagType::DOUBLE: return "double";
    case FlagType::STRING: return "string";
    }
    return "?";
}

std::string to_string_value(const FlagCell& c) {
    switch (c.type) {
    case FlagType::BOOL: return *(bool*)c.storage ? "true" : "false";
    case FlagType::INT32: return std::to_string(*(int32_t*)c.storage);
    case FlagType::INT64: return std::to_string(*(int64_t*)c.storage);
    case FlagType::UINT64: return std::to_string(*(uint64_t*)c.storage);
    case FlagType::DOUBLE: {
        char buf[64];
        snprintf(buf, sizeof(buf), "%g", *(double*)c.storage);
        return buf;
    }
    case FlagType::STRING: return *(std::string*)c.storage;
    }
    return "";
}

// Validates syntax; writes canonical string to *canon.
bool parse_value(FlagType t, const std::string& v, std::string* canon) {
    errno = 0;
    char* end = nullptr;
    switch (t) {
    case FlagType::BOOL:
        if (v == "true" || v == "1" || v == "yes" || v == "on" || v.empty()) { *canon = "true"; return true; }
        if (v == "false" || v == "0" || v == "no" || v == "off") { *canon = "false"; return true; }
        return false;
    case FlagType::INT32: {
        long long x = strtoll(v.c_str(), &end, 0);
        if (errno || end == v.c_str() || *end || x < INT32_MIN || x > INT32_MAX) return false;
        *canon = std::to_string(x);
        return true;
    }
    case FlagType::INT64: {
        long long x = strtoll(v.c_str(), &end, 0);
        if (errno || end == v.c_str() || *end) return false;
        *canon = std::to_string(x);
        return true;
    }
    case FlagType::UINT64: {
        if (!v.empty() && v[0] == '-') return false;
        unsigned long long x = strtoull(v.c_str(), &end, 0);
        if (errno || end == v.c_str() || *end) return false;
        *canon = std::to_string(x);
        return true;
    }
    case FlagType::DOUBLE: {
        strtod(v.c_str(), &end);
        if (errno || end == v.c_str() || *end) return false;
        *canon = v;
        return true;
    }
    case FlagType::STRING:
        *canon = v;
        return true;
    }
    return false;
}

void store_value(FlagCell& c, const std::string& canon) {
    switch (c.type) {
    case FlagType::BOOL: *(bool*)c.storage = (canon == "true"); break;
    case FlagType::INT32: *(int32_t*)c.storage = (int32_t)strtoll(canon.c_str(), nullptr, 0); break;
    case FlagType::INT64: *(int64_t*)c.storage = strtoll(canon.c_str(), nullptr, 0); break;
    case FlagType::UINT64: *(uint64_t*)c.storage = strtoull(canon.c_str(), nullptr, 0); break;
    case FlagType::DOUBLE: *(double*)c.storage = strtod(canon.c_str(), nullptr); break;
    case FlagType::STRING: *(std::string*)c.storage = canon; break;
    }
}
}  // namespace

FlagRegisterer::FlagRegisterer(const char* name, FlagType type, const char* desc, const char* file,
                               void* storage) {
    Registry& r = registry();
    std::lock_guard<std::mutex> g(r.mu);
    FlagCell& c = r.flags[name];
    c.name = name;
    c.type = type;
    c.desc = desc;
    c.file = file;
    c.storage = storage;
    c.default_value = to_string_value(c);
}

bool RegisterFlagValidator(const char* name, FlagValidator v) {
    Registry& r = registry();
    std::lock_guard<std::mutex> g(r.mu);
    auto it = r.flags.find(name);
    if (it == r.flags.end()) {
        // Validators may be registered before the flag in another TU: create
        // a placeholder that the registerer fills in later.
        FlagCell& c = r.flags[name];
        c.name = name;
        c.storage = nullptr;
        c.validator = v;
        c.reloadable = true;
        return true;
    }
    it->second.validator = v;
    it->second.reloadable = true;
    return true;
}

bool SetFlag(const std::string& name, const std::string& value, bool require_reloadable, std::string* error) {
    Registry& r = registry();
    std::lock_guard<std::mutex> g(r.mu);
    auto it = r.flags.find(name);
    if (it == r.flags.end() || it->second.storage == nullptr) {
        if (error) *error = "flag `" + name + "' not found";
        return false;
    }
    FlagCell& c = it->second;
    if (require_reloadable && !c.reloadable) {
        if (error) *error = "flag `" + name + "' is not reloadable";
        return false;
    }
    std::string canon;
    if (!parse_value(c.type, value, &canon)) {
        if (error) *error = "bad value `" + value + "' for " + type_name(c.type) + " flag `" + name + "'";
        return false;
    }
    if (c.validator && !c.validator(name.c_str(), canon)) {
        if (error) *error = "validator rejected `" + value + "' for flag `" + name + "'";
        return false;
    }
    store_value(c, canon);
    return true;
}

bool GetFlag(const std::string& name, std::string* value) {
    Registry& r = registry();
    std::lock_guard<std::mutex> g(r.mu);
    auto it = r.flags.find(name);
    if (it == r.flags.end() || !it->second.storage) return false;
    *value = to_string_value(it->second);
    return true;
}

static FlagInfo make_info(const FlagCell& c) {
    FlagInfo i;
    i.name = c.name;
    i.type = type_name(c.type);
    i.description = c.desc;
    i.file = c.file;
    i.default_value = c.default_value;
    i.current_value = to_string_value(c);
    i.reloadable = c.reloadable;
    return i;
}

bool GetFlagInfo(const std::string& name, FlagInfo* info) {
    Registry& r = registry();
    std::lock_guard<std::mutex> g(r.mu);
    auto it = r.flags.find(name);
    if (it == r.flags.end() || !it->second.storage) return false;
    *info = make_info(it->second);
    return true;
}

std::vector<FlagInfo> ListFlags() {
    Registry& r = registry();
    std::lock_guard<std::mutex> g(r.mu);
    std::vector<FlagInfo> out;
    for (auto& kv : r.flags) {
        if (kv.second.storage) out.push_back(make_info(kv.second));
    }
    return out;
}

int ParseCommandLineFlags(int* argc, char*** argv, bool remove_flags) {
    int applied = 0;
    std::vector<char*> rest;
    rest.push_back((*argv)[0]);
    for (int i = 1; i < *argc; ++i) {
        char* a = (*argv)[i];
        if (a[0] != '-') { rest.push_back(a); continue; }
        const char* s = a + 1;
        if (*s == '-') ++s;
        std::string body(s);
        std::string name, value;
        bool has_value = false;
        size_t eq = body.find('=');
        if (eq != std::string::npos) {
            name = body.substr(0, eq);
            value = body.substr(eq + 1);
            has_value = true;
        } else {
            name = body;
        }
        if (name == "help" || name == "helpfull") {
            // gflags-like: list every flag with its default and exit
            for (const FlagInfo& f : ListFlags()) {
                fprintf(stdout, "  -%s (%s) type: %s default: %s\n", f.name.c_str(), f.description.c_str(),
                        f.type.c_str(), f.default_value.c_str());
            }
            exit(0);
        }
        FlagInfo info;
        bool known = GetFlagInfo(name, &info);
        if (!known && !has_value && name.compare(0, 2, "no") == 0 && GetFlagInfo(name.substr(2), &info) &&
            info.type == "bool") {
            if (!SetFlag(name.substr(2), "false")) return -1;
            ++applied;
            continue;
        }
        if (!known) { rest.push_back(a); continue; }
        if (!has_value) {
            if (info.type == "bool") {
                value = "true";
            } else if (i + 1 < *argc) {
                value = (*argv)[++i];
            } else {
                LOG(ERROR) << "flag --" << name << " needs a value";
                return -1;
            }
        }
        std::string err;
        if (!SetFlag(name, value, false, &err)) {
            LOG(ERROR) << err;
            return -1;
        }
        ++applied;
    }
    if (remove_flags) {
        for (size_t i = 0; i < rest.size(); ++i) (*argv)[i] = rest[i];
        *argc = (int)rest.size();
    }
    return applied;
}

int LoadFlagsFromFile(const std::string& path) {
    std::ifstream in(path);
    if (!in) return -1;
    std::string line;
    int n = 0;
    while (std::getline(in, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();  // CRLF files
        size_t b = line.find_first_not_of(" \t-");
        if (b == std::string::npos || line[b] == '#') continue;
        size_t eq = line.find('=', b);
        if (eq == std::string::npos) continue;
        size_t ne = eq;  // "name = value": the name without trailing blanks
        while (ne > b && (line[ne - 1] == ' ' || line[ne - 1] == '\t')) --ne;
        // ... and the value without blanks on either side ("x = true ")
        size_t vb = eq + 1, ve = line.size();
        while (vb < ve && (line[vb] == ' ' || line[vb] == '\t')) ++vb;
        while (ve > vb && (line[ve - 1] == ' ' || line[ve - 1] == '\t')) --ve;
        if (SetFlag(line.substr(b, ne - b), line.substr(vb, ve - vb))) ++n;
    }
    return n;
}

bool PositiveIntegerValidator(const char*, const std::string& v) { return strtoll(v.c_str(), nullptr, 0) > 0; }
bool NonNegativeIntegerValidator(const char*, const std::string& v) { return strtoll(v.c_str(), nullptr, 0) >= 0; }
bool PassValidator(const char*, const std::string&) { return true; }

}  // namespace mrpc
