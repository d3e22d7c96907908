// A command-line flag seen as a variable (role of the reference's
// bvar/gflag.h: a flag's current value in /vars, the dump file and
// /brpc_metrics, following /flags?setvalue= changes live).
#pragma once

#include <cstdlib>
#include <string>

#include "base/flags.h"
#include "var/variable.h"

namespace mrpc {
namespace var {

class GFlag : public Variable {
public:
    // Exposes flag `flag_name` as variable `flag_name` (or `var_name`).
    explicit GFlag(const std::string& flag_name, const std::string& var_name = std::string()) : _flag(flag_name) {
        expose(var_name.empty() ? flag_name : var_name);
    }
    ~GFlag() override { hide(); }
    const std::string& flag_name() const { return _flag; }
    bool valid() const {
        std::string v;
        return GetFlag(_flag, &v);
    }
    std::string value() const {
        std::string v;
        return GetFlag(_flag, &v) ? v : std::string();
    }
    void describe(std::ostream& os, bool quote_string) const override {
        std::string v;
        if (!GetFlag(_flag, &v)) {
            os << "Unknown flag=" << _flag;
            return;
        }
        if (quote_string && !numeric(v)) os << '"' << v << '"';
        else os << v;
    }
    bool get_number(double* out) const override {
        std::string v;
        if (!GetFlag(_flag, &v)) return false;
        if (v == "true" || v == "false") {
            *out = v == "true";
            return true;
        }
        if (!numeric(v)) return false;
        *out = strtod(v.c_str(), nullptr);
        return true;
    }

private:
    static bool numeric(const std::string& v) {
        if (v.empty()) return false;
        char* end = nullptr;
        strtod(v.c_str(), &end);
        return end && *end == '\0';
    }
    std::string _flag;
};

}  // namespace var
}  // namespace mrpc
