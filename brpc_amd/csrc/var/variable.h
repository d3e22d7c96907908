// Metrics registry (role of bvar/variable.h, reference src/bvar/variable.cpp:
// 463 dump_exposed, 638 prometheus dumper, 698-720 periodic file dump).
// Every metric derives from Variable; exposed variables are visible by name in
// /vars, /brpc_metrics (Prometheus text) and the periodic dump file.
#pragma once

#include <functional>
#include <ostream>
#include <sstream>
#include <string>
#include <vector>

namespace mrpc {
namespace var {

enum DisplayFilter { DISPLAY_ON_HTML = 1, DISPLAY_ON_PLAIN_TEXT = 2, DISPLAY_ON_ALL = 3 };

class Variable {
public:
    Variable() {}
    virtual ~Variable();
    Variable(const Variable&) = delete;
    Variable& operator=(const Variable&) = delete;

    virtual void describe(std::ostream& os, bool quote_string) const = 0;
    // Optional time series for charts (JSON array of [t, v]); empty if none.
    virtual std::string series_json() const { return std::string(); }
    // Numeric value for Prometheus; returns false if not numeric.
    virtual bool get_number(double* out) const;

    // Expose with a normalized name ("a b.c" -> "a_b_c"). Returns 0 on success,
    // -1 if the name is taken.
    int expose(const std::string& name, DisplayFilter f = DISPLAY_ON_ALL) { return expose_impl("", name, f); }
    int expose_as(const std::string& prefix, const std::string& name, DisplayFilter f = DISPLAY_ON_ALL) {
        return expose_impl(prefix, name, f);
    }
    bool hide();
    const std::string& name() const { return _name; }
    bool is_exposed() const { return !_name.empty(); }
    std::string get_description() const;

    static int count_exposed();
    static void list_exposed(std::vector<std::string>* names);
    // Describe by name. Returns -1 if not found.
    static int describe_exposed(const std::string& name, std::ostream& os, bool quote_string = false);
    static std::string describe_exposed(const std::string& name);
    static std::string series_exposed(const std::string& name);
    // name=value lines; `filter` supports wildcards '*' and '?' and ';'
    // separated alternatives ("rpc_*;process_*").
    static int dump_exposed(std::vector<std::pair<std::string, std::string>>* out, const std::string& filter = "",
                            DisplayFilter display = DISPLAY_ON_PLAIN_TEXT);
    static std::string dump_prometheus();

protected:
    int expose_impl(const std::string& prefix, const std::string& name, DisplayFilter f);

private:
    std::string _name;
};

std::string normalize_name(const std::string& s);
bool wildcard_match(const std::string& pattern, const std::string& s);

// Start the periodic dump thread (flag var_dump / var_dump_file / var_dump_interval).
void start_dump_thread_if_needed();

}  // namespace var
}  // namespace mrpc
