// Flag registry with runtime ("reloadable") updates.
//
// The reference relies on gflags (205 DEFINE_* in src/) plus
// BRPC_VALIDATE_GFLAG (reference src/brpc/reloadable_flags.h:25-71) to mark
// flags as settable through /flags?setvalue= (builtin/flags_service.cpp:150).
// gflags is not available here, so this is a self-contained registry: every
// DEFINE_* registers a typed cell; MRPC_VALIDATE_FLAG attaches a validator and
// makes the flag reloadable at runtime.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace mrpc {

enum class FlagType { BOOL, INT32, INT64, UINT64, DOUBLE, STRING };

struct FlagInfo {
    std::string name;
    std::string type;
    std::string description;
    std::string file;
    std::string default_value;
    std::string current_value;
    bool reloadable;
};

class FlagRegisterer {
public:
    FlagRegisterer(const char* name, FlagType type, const char* desc, const char* file, void* storage);
};

// Validator receives the *new* value in string form already converted and
// returns false to reject it.
using FlagValidator = std::function<bool(const char* name, const std::string& new_value)>;
bool RegisterFlagValidator(const char* name, FlagValidator v);

// Returns false if not found / bad value / validator rejected / not reloadable
// (when require_reloadable is true).
bool SetFlag(const std::string& name, const std::string& value, bool require_reloadable = false,
             std::string* error = nullptr);
bool GetFlag(const std::string& name, std::string* value);
bool GetFlagInfo(const std::string& name, FlagInfo* info);
std::vector<FlagInfo> ListFlags();
// Consumes --name=value / -name=value / --name value / --noname arguments
// that match registered flags. Unknown flags are left in argv. Returns the
// number of flags applied, or -1 on a bad value.
int ParseCommandLineFlags(int* argc, char*** argv, bool remove_flags = true);
// Reads name=value lines (a --flagfile analog).
int LoadFlagsFromFile(const std::string& path);

// Helpers for validators of positive numbers.
bool PositiveIntegerValidator(const char*, const std::string& v);
bool NonNegativeIntegerValidator(const char*, const std::string& v);
bool PassValidator(const char*, const std::string&);

}  // namespace mrpc

#define MRPC_DEFINE_FLAG_(ctype, ftype, name, defval, desc) \
    ctype FLAGS_##name = defval;                            \
    static ::mrpc::FlagRegisterer _mrpc_flag_reg_##name(#name, ::mrpc::FlagType::ftype, desc, __FILE__, &FLAGS_##name)

#define DEFINE_bool(name, defval, desc) MRPC_DEFINE_FLAG_(bool, BOOL, name, defval, desc)
#define DEFINE_int32(name, defval, desc) MRPC_DEFINE_FLAG_(int32_t, INT32, name, defval, desc)
#define DEFINE_int64(name, defval, desc) MRPC_DEFINE_FLAG_(int64_t, INT64, name, defval, desc)
#define DEFINE_uint64(name, defval, desc) MRPC_DEFINE_FLAG_(uint64_t, UINT64, name, defval, desc)
#define DEFINE_double(name, defval, desc) MRPC_DEFINE_FLAG_(double, DOUBLE, name, defval, desc)
#define DEFINE_string(name, defval, desc) MRPC_DEFINE_FLAG_(std::string, STRING, name, defval, desc)

#define DECLARE_bool(name) extern bool FLAGS_##name
#define DECLARE_int32(name) extern int32_t FLAGS_##name
#define DECLARE_int64(name) extern int64_t FLAGS_##name
#define DECLARE_uint64(name) extern uint64_t FLAGS_##name
#define DECLARE_double(name) extern double FLAGS_##name
#define DECLARE_string(name) extern std::string FLAGS_##name

// Marks a flag reloadable at runtime with a validator.
#define MRPC_VALIDATE_FLAG(name, fn) \
    static const bool _mrpc_flag_validate_##name = ::mrpc::RegisterFlagValidator(#name, fn)
