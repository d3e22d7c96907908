// IntRecorder (average of recorded ints, role of bvar/recorder.h:84),
// PassiveStatus (callback-backed, passive_status.h:42), Status (settable,
// status.h:44), and MultiDimension (labelled families, multi_dimension.h:35).
#pragma once


#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "var/reducer.h"
#include "var/window.h"

namespace mrpc {
namespace var {

struct Stat {
    int64_t sum = 0;
    int64_t num = 0;
    double average() const { return num ? (double)sum / num : 0.0; }
    int64_t get_average_int() const { return num ? sum / num : 0; }
};

class IntRecorder : public Variable {
public:
    IntRecorder() {}
    explicit IntRecorder(const std::string& name) { expose(name); }
    IntRecorder& operator<<(int64_t v) {
        _sum << v;
        _num << 1;
        return *this;
    }
    Stat get_value() const {
        Stat s;
        s.sum = _sum.get_value();
        s.num = _num.get_value();
        return s;
    }
    void describe(std::ostream& os, bool) const override { os << get_value().get_average_int(); }
    bool get_number(double* out) const override {
        *out = get_value().average();
        return true;
    }
    Adder<int64_t>* sum_adder() { return &_sum; }
    Adder<int64_t>* num_adder() { return &_num; }

private:
    Adder<int64_t> _sum;
    Adder<int64_t> _num;
};

// Average of an IntRecorder over a window.
class IntRecorderWindow : public Variable {
public:
    IntRecorderWindow(IntRecorder* r, int window) : _s(r->sum_adder(), window < 60 ? 60 : window),
                                                    _n(r->num_adder(), window < 60 ? 60 : window), _w(window) {
        _s.schedule();
        _n.schedule();
    }
    ~IntRecorderWindow() {
        hide();
        _s.unschedule();
        _n.unschedule();
    }
    Stat get_value() const {
        Stat st;
        st.sum = _s.value_over(_w, nullptr);
        st.num = _n.value_over(_w, nullptr);
        return st;
    }
    void describe(std::ostream& os, bool) const override { os << get_value().get_average_int(); }
    bool get_number(double* out) const override {
        *out = get_value().average();
        return true;
    }

private:
    ReducerSampler<Adder<int64_t>> _s;
    ReducerSampler<Adder<int64_t>> _n;
    int _w;
};

template <typename T>
class PassiveStatus : public Variable {
public:
    typedef std::function<T()> Getter;
    explicit PassiveStatus(Getter g) : _g(std::move(g)) {}
    PassiveStatus(const std::string& name, Getter g) : _g(std::move(g)) { expose(name); }
    PassiveStatus(const std::string& prefix, const std::string& name, Getter g) : _g(std::move(g)) {
        expose_as(prefix, name);
    }
    ~PassiveStatus() { hide(); }
    T get_value() const { return _g ? _g() : T(); }
    void describe(std::ostream& os, bool quote) const override {
        if constexpr (std::is_same<T, std::string>::value) {
            if (quote) os << '"' << get_value() << '"';
            else os << get_value();
        } else {
            os << get_value();
        }
    }
    bool get_number(double* out) const override {
        if constexpr (std::is_arithmetic<T>::value) {
            *out = (double)get_value();
            return true;
        } else {
            return false;
        }
    }

private:
    Getter _g;
};

template <typename T>
class Status : public Variable {
public:
    Status() : _v() {}
    explicit Status(const T& v) : _v(v) {}
    Status(const std::string& name, const T& v) : _v(v) { expose(name); }
    ~Status() { hide(); }
    void set_value(const T& v) {
        std::lock_guard<std::mutex> g(_mu);
        _v = v;
    }
    T get_value() const {
        std::lock_guard<std::mutex> g(_mu);
        return _v;
    }
    void describe(std::ostream& os, bool quote) const override {
        T v = get_value();
        if constexpr (std::is_same<T, std::string>::value) {
            if (quote) os << '"' << v << '"';
            else os << v;
        } else {
            os << v;
        }
    }
    bool get_number(double* out) const override {
        if constexpr (std::is_arithmetic<T>::value) {
            *out = (double)get_value();
            return true;
        } else {
            return false;
        }
    }

private:
    mutable std::mutex _mu;
    T _v;
};

// Registers process-level variables (cpu, memory, fds, io, loadavg, uptime)
// read from /proc (role of bvar/default_variables.cpp:128-691).
void ExposeDefaultVariables();

}  // namespace var
}  // namespace mrpc
