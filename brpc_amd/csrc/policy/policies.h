// Registration entry points of all built-in protocols (called from
// GlobalInitializeOrDie, role of reference global.cpp:356-606).
#pragma once

namespace mrpc {
namespace policy {

void RegisterBaiduStdProtocol();
void RegisterHttpProtocol();
void RegisterH2Protocol();
void RegisterRedisProtocol();
void RegisterMemcacheProtocol();
void RegisterHuluProtocol();
void RegisterSofaProtocol();
void RegisterNovaProtocol();
void RegisterPublicPbrpcProtocol();
void RegisterNsheadProtocols();
void RegisterEspProtocol();
void RegisterMongoProtocol();
void RegisterThriftProtocol();
void RegisterUbrpcProtocols();
void RegisterRtmpProtocol();

}  // namespace policy
}  // namespace mrpc
