// .proto parser + importer (proto2/proto3). Builds descriptors (with
// dynamic layouts) for runtime loading — rpc_press / rpc_replay load .proto
// files at runtime like the reference does with compiler::Importer
// (tools/rpc_press/rpc_press_impl.cpp) — and for the code generator
// (tools/protoc_main.cc). No protoc exists in this environment.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "pb/descriptor.h"

namespace mrpc {
namespace pb {

class Importer {
public:
    explicit Importer(const std::vector<std::string>& proto_paths);
    ~Importer();
    // Loads `filename` (relative to a proto path) and its imports. Returns
    // nullptr and fills *error on failure.
    const FileDescriptor* Import(const std::string& filename, std::string* error);
    // Parse from memory (name is used for imports bookkeeping).
    const FileDescriptor* ImportFromString(const std::string& name, const std::string& content, std::string* error);
    DescriptorPool* pool() { return _pool.get(); }
    const Descriptor* FindMessageTypeByName(const std::string& n) const { return _pool->FindMessageTypeByName(n); }
    const ServiceDescriptor* FindServiceByName(const std::string& n) const { return _pool->FindServiceByName(n); }
    const MethodDescriptor* FindMethodByName(const std::string& n) const { return _pool->FindMethodByName(n); }

private:
    const FileDescriptor* load(const std::string& filename, std::string* error, int depth);
    bool read_source(const std::string& filename, std::string* content);
    std::vector<std::string> _paths;
    std::unique_ptr<DescriptorPool> _pool;
    std::map<std::string, const FileDescriptor*> _loaded;
};

// Lower-level: parse one file's text into an unresolved FileDescriptor.
// Type references are resolved by Importer.
FileDescriptor* ParseProtoText(const std::string& filename, const std::string& text, std::string* error);

}  // namespace pb
}  // namespace mrpc
