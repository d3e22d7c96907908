// protobuf <-> JSON conversion over descriptor reflection (role of
// src/json2pb/json_to_pb.h:54-88, pb_to_json.h:76-90). Works for generated
// and dynamic messages: rpc_press inputs, http+json bodies, /protobufs.
#pragma once

#include <string>
#include <vector>

#include "base/buf.h"
#include "json/json.h"
#include "pb/message.h"

namespace mrpc {
namespace json2pb {

struct Pb2JsonOptions {
    bool enum_option_as_string = true;  // else as number
    bool pretty_json = false;
    bool bytes_to_base64 = true;
    bool jsonify_empty_array = false;
    bool always_print_primitive_fields = false;
    bool use_json_name = false;  // camelCase keys
};

struct Json2PbOptions {
    bool base64_to_bytes = true;
    bool allow_unknown_fields = true;
};

bool ProtoMessageToJson(const pb::Message& msg, std::string* json, const Pb2JsonOptions& opt = Pb2JsonOptions(),
                        std::string* error = nullptr);
bool ProtoMessageToJsonValue(const pb::Message& msg, json::Value* out, const Pb2JsonOptions& opt, std::string* error);
bool JsonToProtoMessage(const std::string& json, pb::Message* msg, const Json2PbOptions& opt = Json2PbOptions(),
                        std::string* error = nullptr);
bool JsonToProtoMessage(const Buf& json, pb::Message* msg, const Json2PbOptions& opt = Json2PbOptions(),
                        std::string* error = nullptr);
bool JsonValueToProtoMessage(const json::Value& v, pb::Message* msg, const Json2PbOptions& opt, std::string* error);

// Hook for a structural index of large bodies built on the GPU
// (gpu/json_offload.cc, kernel K6): fills *index for data[0, n) and returns
// true, or false to parse without one. Bodies of at least min_bytes use it.
// pb2json of large repeated integer/bool fields: the offload
// prints the numbers of one field — values in the field's vector layout,
// kind a gpu PbRunKind — as "v,v,...,v" into *text (false: the host prints
// them). Only for compact output (not pretty_json) and fields of at least
// min_elems elements; enums printed as names stay on the host.
typedef bool (*Pb2JsonArrayOffload)(const void* values, size_t n, uint32_t kind, std::string* text);
void SetPb2JsonArrayOffload(Pb2JsonArrayOffload fn, size_t min_elems);
typedef bool (*JsonIndexOffload)(const char* data, size_t n, std::vector<uint32_t>* index);
void SetJsonIndexOffload(JsonIndexOffload fn, size_t min_bytes);

}  // namespace json2pb
}  // namespace mrpc
