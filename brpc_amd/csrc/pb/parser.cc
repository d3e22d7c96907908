#include "pb/parser.h"

#include <cctype>
#include <cstdlib>
#include <fstream>
#include <functional>
#include <sstream>

#include "pb/dynamic.h"

namespace mrpc {
namespace pb {

namespace {

// Minimal well-known types so that common imports resolve without files.
const char* kBuiltinFiles[][2] = {
    {"google/protobuf/descriptor.proto", "syntax = \"proto2\"; package google.protobuf;"},
    {"google/protobuf/empty.proto", "syntax = \"proto3\"; package google.protobuf; message Empty {}"},
    {"google/protobuf/timestamp.proto",
     "syntax = \"proto3\"; package google.protobuf; message Timestamp { int64 seconds = 1; int32 nanos = 2; }"},
    {"google/protobuf/duration.proto",
     "syntax = \"proto3\"; package google.protobuf; message Duration { int64 seconds = 1; int32 nanos = 2; }"},
    {"google/protobuf/any.proto",
     "syntax = \"proto3\"; package google.protobuf; message Any { string type_url = 1; bytes value = 2; }"},
    {"google/protobuf/wrappers.proto",
     "syntax = \"proto3\"; package google.protobuf;"
     "message DoubleValue { double value = 1; } message FloatValue { float value = 1; }"
     "message Int64Value { int64 value = 1; } message UInt64Value { uint64 value = 1; }"
     "message Int32Value { int32 value = 1; } message UInt32Value { uint32 value = 1; }"
     "message BoolValue { bool value = 1; } message StringValue { string value = 1; }"
     "message BytesValue { bytes value = 1; }"},
};

enum TokType { T_END, T_IDENT, T_INT, T_FLOAT, T_STRING, T_SYMBOL };

struct Token {
    TokType type = T_END;
    std::string text;
    int line = 0;
};

class Tokenizer {
public:
    explicit Tokenizer(const std::string& s) : _s(s), _i(0), _line(1) { advance(); }
    const Token& cur() const { return _cur; }
    void advance() { _cur = next(); }

private:
    Token next() {
        skip_ws();
        Token t;
        t.line = _line;
        if (_i >= _s.size()) return t;
        char c = _s[_i];
        if (isalpha((unsigned char)c) || c == '_') {
            size_t b = _i;
            while (_i < _s.size() && (isalnum((unsigned char)_s[_i]) || _s[_i] == '_' || _s[_i] == '.')) ++_i;
            t.type = T_IDENT;
            t.text = _s.substr(b, _i - b);
            return t;
        }
        if (isdigit((unsigned char)c) || (c == '.' && _i + 1 < _s.size() && isdigit((unsigned char)_s[_i + 1]))) {
            size_t b = _i;
            bool is_float = false;
            if (c == '0' && _i + 1 < _s.size() && (_s[_i + 1] == 'x' || _s[_i + 1] == 'X')) {
                _i += 2;
                while (_i < _s.size() && isxdigit((unsigned char)_s[_i])) ++_i;
            } else {
                while (_i < _s.size() && (isalnum((unsigned char)_s[_i]) || _s[_i] == '.' ||
                                          ((_s[_i] == '-' || _s[_i] == '+') && (_s[_i - 1] == 'e' || _s[_i - 1] == 'E')))) {
                    if (_s[_i] == '.' || _s[_i] == 'e' || _s[_i] == 'E') is_float = true;
                    ++_i;
                }
            }
            t.type = is_float ? T_FLOAT : T_INT;
            t.text = _s.substr(b, _i - b);
            return t;
        }
        if (c == '"' || c == '\'') {
            t.type = T_STRING;
            // adjacent string literals concatenate
            for (;;) {
                char q = _s[_i++];
                while (_i < _s.size() && _s[_i] != q) {
                    char ch = _s[_i++];
                    if (ch == '\\' && _i < _s.size()) {
                        char e = _s[_i++];
                        switch (e) {
                        case 'n': t.text.push_back('\n'); break;
                        case 't': t.text.push_back('\t'); break;
                        case 'r': t.text.push_back('\r'); break;
                        case '0': case '1': case '2': case '3': case '4': case '5': case '6': case '7': {
                            int v = e - '0';
                            for (int k = 0; k < 2 && _i < _s.size() && _s[_i] >= '0' && _s[_i] <= '7'; ++k) v = v * 8 + (_s[_i++] - '0');
                            t.text.push_back((char)v);
                            break;
                        }
                        case 'x': {
                            int v = 0;
                            for (int k = 0; k < 2 && _i < _s.size() && isxdigit((unsigned char)_s[_i]); ++k) {
                                char h = _s[_i++];
                                v = v * 16 + (isdigit((unsigned char)h) ? h - '0' : (tolower(h) - 'a' + 10));
                            }
                            t.text.push_back((char)v);
                            break;
                        }
                        default: t.text.push_back(e);
                        }
                    } else {
                        if (ch == '\n') ++_line;
                        t.text.push_back(ch);
                    }
                }
                ++_i;  // closing quote
                skip_ws();
                if (_i < _s.size() && (_s[_i] == '"' || _s[_i] == '\'')) continue;
                break;
            }
            return t;
        }
        t.type = T_SYMBOL;
        t.text = std::string(1, c);
        ++_i;
        return t;
    }
    void skip_ws() {
        for (;;) {
            while (_i < _s.size() && isspace((unsigned char)_s[_i])) {
                if (_s[_i] == '\n') ++_line;
                ++_i;
            }
            if (_i + 1 < _s.size() && _s[_i] == '/' && _s[_i + 1] == '/') {
                while (_i < _s.size() && _s[_i] != '\n') ++_i;
                continue;
            }
            if (_i + 1 < _s.size() && _s[_i] == '/' && _s[_i + 1] == '*') {
                _i += 2;
                while (_i + 1 < _s.size() && !(_s[_i] == '*' && _s[_i + 1] == '/')) {
                    if (_s[_i] == '\n') ++_line;
                    ++_i;
                }
                _i += 2;
                continue;
            }
            break;
        }
    }
    const std::string& _s;
    size_t _i;
    int _line;
    Token _cur;
};

struct ParseError {
    std::string msg;
};

class Parser {
public:
    Parser(const std::string& filename, const std::string& text) : _tok(text), _filename(filename) {}

    FileDescriptor* parse() {
        _file = new FileDescriptor;
        _file->name = _filename;
        try {
            while (_tok.cur().type != T_END) parse_top();
        } catch (ParseError& e) {
            delete_file();
            _error = e.msg;
            return nullptr;
        }
        return _file;
    }
    const std::string& error() const { return _error; }

private:
    void delete_file() {
        delete _file;  // frees every descriptor parsed so far (owned_*)
        _file = nullptr;
    }
    [[noreturn]] void fail(const std::string& what) {
        std::ostringstream os;
        os << _filename << ":" << _tok.cur().line << ": " << what << " (near '" << _tok.cur().text << "')";
        throw ParseError{os.str()};
    }
    bool is(const char* sym) const { return _tok.cur().text == sym && (_tok.cur().type == T_SYMBOL || _tok.cur().type == T_IDENT); }
    void expect(const char* sym) {
        if (_tok.cur().text != sym) fail(std::string("expected '") + sym + "'");
        _tok.advance();
    }
    bool accept(const char* sym) {
        if (_tok.cur().text == sym && _tok.cur().type != T_STRING) {
            _tok.advance();
            return true;
        }
        return false;
    }
    std::string ident() {
        if (_tok.cur().type != T_IDENT) fail("expected identifier");
        std::string s = _tok.cur().text;
        _tok.advance();
        return s;
    }
    // type name possibly starting with '.'
    std::string type_ref() {
        std::string s;
        if (accept(".")) s = ".";
        s += ident();
        return s;
    }
    std::string string_lit() {
        if (_tok.cur().type != T_STRING) fail("expected string");
        std::string s = _tok.cur().text;
        _tok.advance();
        return s;
    }
    int64_t int_lit() {
        bool neg = accept("-");
        if (_tok.cur().type != T_INT) fail("expected integer");
        int64_t v = (int64_t)strtoull(_tok.cur().text.c_str(), nullptr, 0);
        _tok.advance();
        return neg ? -v : v;
    }
    // option value: identifier, number, string, or aggregate {...}
    std::string option_value() {
        std::string v;
        if (accept("-")) v = "-";
        const Token& t = _tok.cur();
        if (t.type == T_STRING || t.type == T_INT || t.type == T_FLOAT || t.type == T_IDENT) {
            v += t.text;
            _tok.advance();
            return v;
        }
        if (is("{")) {
            int depth = 0;
            do {
                if (is("{")) ++depth;
                else if (is("}")) --depth;
                v += _tok.cur().text + " ";
                _tok.advance();
            } while (depth > 0 && _tok.cur().type != T_END);
            return v;
        }
        fail("bad option value");
    }
    std::string option_name() {
        std::string n;
        if (accept("(")) {
            n = "(" + type_ref() + ")";
            expect(")");
        } else {
            n = ident();
        }
        while (_tok.cur().type == T_IDENT && _tok.cur().text[0] == '.') {
            n += _tok.cur().text;
            _tok.advance();
        }
        return n;
    }
    void option_statement(std::map<std::string, std::string>* opts) {
        // after 'option'
        std::string name = option_name();
        expect("=");
        (*opts)[name] = option_value();
        expect(";");
    }
    void field_options(std::map<std::string, std::string>* opts) {
        if (!accept("[")) return;
        do {
            std::string name = option_name();
            expect("=");
            (*opts)[name] = option_value();
        } while (accept(","));
        expect("]");
    }
    void skip_statement_or_block() {
        int depth = 0;
        while (_tok.cur().type != T_END) {
            if (is("{")) ++depth;
            if (is("}")) {
                --depth;
                if (depth <= 0) {
                    _tok.advance();
                    return;
                }
            }
            if (is(";") && depth == 0) {
                _tok.advance();
                return;
            }
            _tok.advance();
        }
    }
    std::string scope_prefix(const std::string& scope) const { return scope.empty() ? "" : scope + "."; }

    void parse_top() {
        if (accept(";")) return;
        if (accept("syntax")) {
            expect("=");
            _file->syntax = string_lit();
            expect(";");
            return;
        }
        if (accept("package")) {
            _file->package = ident();
            expect(";");
            return;
        }
        if (accept("import")) {
            if (is("public") || is("weak")) _tok.advance();
            _file->dependencies.push_back(string_lit());
            expect(";");
            return;
        }
        if (accept("option")) {
            option_statement(&_file->options);
            return;
        }
        if (accept("message")) {
            _file->message_types.push_back(parse_message(_file->package, nullptr));
            return;
        }
        if (accept("enum")) {
            _file->enum_types.push_back(parse_enum(_file->package));
            return;
        }
        if (accept("service")) {
            _file->services.push_back(parse_service());
            return;
        }
        if (accept("extend")) {
            type_ref();
            skip_statement_or_block();
            return;
        }
        fail("unexpected token at top level");
    }

    EnumDescriptor* parse_enum(const std::string& scope) {
        EnumDescriptor* e = new EnumDescriptor;
        _file->owned_enums.emplace_back(e);
        e->name = ident();
        e->full_name = scope_prefix(scope) + e->name;
        e->file = _file;
        expect("{");
        while (!accept("}")) {
            if (accept(";")) continue;
            if (accept("option")) {
                std::map<std::string, std::string> o;
                option_statement(&o);
                continue;
            }
            if (accept("reserved")) {
                skip_statement_or_block();
                continue;
            }
            EnumValueDescriptor v;
            v.name = ident();
            expect("=");
            v.number = (int)int_lit();
            std::map<std::string, std::string> o;
            field_options(&o);
            expect(";");
            e->values.push_back(v);
        }
        return e;
    }

    FieldType scalar_type(const std::string& t, bool* is_scalar) {
        static const std::map<std::string, FieldType> m = {
            {"double", FieldType::DOUBLE}, {"float", FieldType::FLOAT}, {"int64", FieldType::INT64},
            {"uint64", FieldType::UINT64}, {"int32", FieldType::INT32}, {"fixed64", FieldType::FIXED64},
            {"fixed32", FieldType::FIXED32}, {"bool", FieldType::BOOL}, {"string", FieldType::STRING},
            {"bytes", FieldType::BYTES}, {"uint32", FieldType::UINT32}, {"sfixed32", FieldType::SFIXED32},
            {"sfixed64", FieldType::SFIXED64}, {"sint32", FieldType::SINT32}, {"sint64", FieldType::SINT64},
        };
        auto it = m.find(t);
        *is_scalar = it != m.end();
        return *is_scalar ? it->second : FieldType::MESSAGE;
    }

    void finish_field(FieldDescriptor& f, const std::string& type, bool proto3, bool explicit_optional,
                      std::map<std::string, std::string>& opts) {
        bool scalar;
        f.type = scalar_type(type, &scalar);
        if (!scalar) {
            f.type = FieldType::MESSAGE;  // may become ENUM at resolution
            f.type_name = type;
        }
        f.options = opts;
        auto it = opts.find("default");
        if (it != opts.end()) {
            f.has_default = true;
            f.default_str = it->second;
        }
        it = opts.find("json_name");
        if (it != opts.end()) f.json_name = it->second;
        if (f.is_repeated()) {
            it = opts.find("packed");
            if (it != opts.end()) f.packed = (it->second == "true");
            else f.packed = proto3 && scalar && f.type != FieldType::STRING && f.type != FieldType::BYTES;
        }
        if (proto3 && !f.is_repeated() && !explicit_optional && f.oneof_index < 0) f.proto3_implicit = true;
    }

    Descriptor* parse_message(const std::string& scope, Descriptor* parent) {
        Descriptor* d = new Descriptor;
        _file->owned_messages.emplace_back(d);
        d->name = ident();
        d->full_name = scope_prefix(scope) + d->name;
        d->file = _file;
        d->containing_type = parent;
        d->proto3 = (_file->syntax == "proto3");
        expect("{");
        parse_message_body(d, -1);
        return d;
    }

    void parse_message_body(Descriptor* d, int oneof_index) {
        const bool proto3 = d->proto3;
        while (!accept("}")) {
            if (accept(";")) continue;
            if (oneof_index < 0) {
                if (accept("message")) {
                    d->nested_types.push_back(parse_message(d->full_name, d));
                    continue;
                }
                if (accept("enum")) {
                    d->enum_types.push_back(parse_enum(d->full_name));
                    continue;
                }
                if (accept("oneof")) {
                    int idx = (int)d->oneof_names.size();
                    d->oneof_names.push_back(ident());
                    expect("{");
                    parse_message_body(d, idx);
                    continue;
                }
                if (accept("extensions") || accept("reserved")) {
                    skip_statement_or_block();
                    continue;
                }
                if (accept("extend")) {
                    type_ref();
                    skip_statement_or_block();
                    continue;
                }
            }
            if (accept("option")) {
                std::map<std::string, std::string> o;
                option_statement(&o);
                continue;
            }
            FieldDescriptor f;
            f.oneof_index = oneof_index;
            bool explicit_optional = false;
            if (accept("optional")) {
                f.label = Label::OPTIONAL;
                explicit_optional = true;
            } else if (accept("required")) {
                f.label = Label::REQUIRED;
            } else if (accept("repeated")) {
                f.label = Label::REPEATED;
            }
            if (accept("map")) {
                expect("<");
                std::string kt = type_ref();
                expect(",");
                std::string vt = type_ref();
                expect(">");
                f.name = ident();
                expect("=");
                f.number = (int)int_lit();
                std::map<std::string, std::string> opts;
                field_options(&opts);
                expect(";");
                // synthesize the entry type
                Descriptor* e = new Descriptor;
                _file->owned_messages.emplace_back(e);
                std::string camel;
                bool up = true;
                for (char c : f.name) {
                    if (c == '_') {
                        up = true;
                        continue;
                    }
                    camel.push_back(up ? (char)toupper((unsigned char)c) : c);
                    up = false;
                }
                e->name = camel + "Entry";
                e->full_name = d->full_name + "." + e->name;
                e->file = _file;
                e->containing_type = d;
                e->map_entry = true;
                e->proto3 = proto3;
                FieldDescriptor kf, vf;
                std::map<std::string, std::string> none;
                kf.name = "key";
                kf.number = 1;
                finish_field(kf, kt, false, true, none);
                vf.name = "value";
                vf.number = 2;
                finish_field(vf, vt, false, true, none);
                e->fields.push_back(kf);
                e->fields.push_back(vf);
                d->nested_types.push_back(e);
                f.label = Label::REPEATED;
                f.type = FieldType::MESSAGE;
                f.type_name = e->full_name;
                f.type_name.insert(0, ".");
                f.options = opts;
                d->fields.push_back(f);
                continue;
            }
            if (accept("group")) fail("groups are not supported");
            std::string type = type_ref();
            f.name = ident();
            expect("=");
            f.number = (int)int_lit();
            std::map<std::string, std::string> opts;
            field_options(&opts);
            expect(";");
            finish_field(f, type, proto3, explicit_optional, opts);
            d->fields.push_back(f);
        }
    }

    ServiceDescriptor* parse_service() {
        ServiceDescriptor* s = new ServiceDescriptor;
        _file->owned_services.emplace_back(s);
        s->name = ident();
        s->full_name = scope_prefix(_file->package) + s->name;
        s->file = _file;
        expect("{");
        while (!accept("}")) {
            if (accept(";")) continue;
            if (accept("option")) {
                option_statement(&s->options);
                continue;
            }
            if (!accept("rpc")) fail("expected rpc");
            MethodDescriptor m;
            m.name = ident();
            m.full_name = s->full_name + "." + m.name;
            expect("(");
            if (is("stream")) {
                _tok.advance();
                m.client_streaming = true;
            }
            m.input_type_name = type_ref();
            expect(")");
            expect("returns");
            expect("(");
            if (is("stream")) {
                _tok.advance();
                m.server_streaming = true;
            }
            m.output_type_name = type_ref();
            expect(")");
            if (accept("{")) {
                while (!accept("}")) {
                    if (accept(";")) continue;
                    if (accept("option")) option_statement(&m.options);
                    else fail("expected option in rpc body");
                }
            } else {
                expect(";");
            }
            m.index = (int)s->methods.size();
            s->methods.push_back(m);
        }
        for (auto& m : s->methods) m.service = s;
        return s;
    }

    Tokenizer _tok;
    std::string _filename;
    FileDescriptor* _file = nullptr;
    std::string _error;
};

// Resolve a possibly-relative type name in `scope`.
template <typename LookupFn>
auto resolve_name(const std::string& name, const std::string& scope, LookupFn lookup) -> decltype(lookup(name)) {
    if (!name.empty() && name[0] == '.') return lookup(name.substr(1));
    std::string s = scope;
    for (;;) {
        auto r = lookup(s.empty() ? name : s + "." + name);
        if (r) return r;
        if (s.empty()) break;
        size_t dot = s.rfind('.');
        s = dot == std::string::npos ? "" : s.substr(0, dot);
    }
    return nullptr;
}

bool resolve_message(Descriptor* d, DescriptorPool* pool, std::string* error) {
    for (Descriptor* n : d->nested_types) {
        if (!resolve_message(n, pool, error)) return false;
    }
    for (FieldDescriptor& f : d->fields) {
        if (f.type_name.empty()) continue;
        const Descriptor* md = resolve_name(f.type_name, d->full_name,
                                            [pool](const std::string& n) { return pool->FindMessageTypeByName(n); });
        if (md) {
            f.type = FieldType::MESSAGE;
            f.message_type = md;
            f.type_name = "." + md->full_name;
            f.proto3_implicit = false;
            f.packed = false;
            continue;
        }
        const EnumDescriptor* ed = resolve_name(f.type_name, d->full_name,
                                                [pool](const std::string& n) { return pool->FindEnumTypeByName(n); });
        if (ed) {
            f.type = FieldType::ENUM;
            f.enum_type = ed;
            f.type_name = "." + ed->full_name;
            if (f.is_repeated() && d->proto3 && f.options.find("packed") == f.options.end()) f.packed = true;
            continue;
        }
        *error = d->file->name + ": unresolved type '" + f.type_name + "' in " + d->full_name;
        return false;
    }
    for (FieldDescriptor& f : d->fields) ResolveDefaultValue(&f);
    d->BuildIndex();
    return true;
}

}  // namespace

FileDescriptor* ParseProtoText(const std::string& filename, const std::string& text, std::string* error) {
    Parser p(filename, text);
    FileDescriptor* f = p.parse();
    if (!f && error) *error = p.error();
    if (f) f->source = text;
    return f;
}

Importer::Importer(const std::vector<std::string>& proto_paths) : _paths(proto_paths), _pool(new DescriptorPool) {
    if (_paths.empty()) _paths.push_back(".");
}

Importer::~Importer() {}

bool Importer::read_source(const std::string& filename, std::string* content) {
    for (auto& b : kBuiltinFiles) {
        if (filename == b[0]) {
            *content = b[1];
            return true;
        }
    }
    for (const std::string& p : _paths) {
        std::ifstream in(p + "/" + filename);
        if (!in) continue;
        std::stringstream ss;
        ss << in.rdbuf();
        *content = ss.str();
        return true;
    }
    std::ifstream in(filename);
    if (in) {
        std::stringstream ss;
        ss << in.rdbuf();
        *content = ss.str();
        return true;
    }
    return false;
}

const FileDescriptor* Importer::ImportFromString(const std::string& name, const std::string& content, std::string* error) {
    auto it = _loaded.find(name);
    if (it != _loaded.end()) return it->second;
    std::string err;
    FileDescriptor* f = ParseProtoText(name, content, &err);
    if (!f) {
        if (error) *error = err;
        return nullptr;
    }
    for (const std::string& dep : f->dependencies) {
        if (!load(dep, error, 1)) return nullptr;
    }
    _pool->AddFile(f);
    _loaded[name] = f;
    for (Descriptor* d : f->message_types) {
        if (!resolve_message(d, _pool.get(), &err)) {
            if (error) *error = err;
            return nullptr;
        }
    }
    for (ServiceDescriptor* s : f->services) {
        for (MethodDescriptor& m : s->methods) {
            auto lk = [this](const std::string& n) { return _pool->FindMessageTypeByName(n); };
            m.input_type = resolve_name(m.input_type_name, f->package, lk);
            m.output_type = resolve_name(m.output_type_name, f->package, lk);
            if (!m.input_type || !m.output_type) {
                if (error) *error = name + ": unresolved request/response type of " + m.full_name;
                return nullptr;
            }
        }
    }
    for (Descriptor* d : f->message_types) PrepareDynamicLayout(d);
    return f;
}

const FileDescriptor* Importer::load(const std::string& filename, std::string* error, int depth) {
    if (depth > 64) {
        if (error) *error = "import depth exceeded at " + filename;
        return nullptr;
    }
    auto it = _loaded.find(filename);
    if (it != _loaded.end()) return it->second;
    std::string content;
    if (!read_source(filename, &content)) {
        if (error) *error = "cannot open " + filename;
        return nullptr;
    }
    return ImportFromString(filename, content, error);
}

const FileDescriptor* Importer::Import(const std::string& filename, std::string* error) {
    return load(filename, error, 0);
}

}  // namespace pb
}  // namespace mrpc
