#include "rpc/ordered_response.h"

#include "base/logging.h"
#include "net/socket.h"

namespace mrpc {

void OrderedResponseWriter::Deliver(uint64_t seq, Buf* packet, Socket* sock) {
    Buf out;
    {
        std::lock_guard<fiber::Mutex> g(_mu);
        if (seq != _next_send) {
            _ready[seq].swap(*packet);
            return;
        }
        out.swap(*packet);
        ++_next_send;
        for (auto it = _ready.begin(); it != _ready.end() && it->first == _next_send; it = _ready.erase(it)) {
            out.append(std::move(it->second));
            ++_next_send;
        }
        // Write under the lock so that batches of consecutive deliverers
        // cannot overtake each other.
        if (!out.empty()) {
            WriteOptions wopt;
            wopt.ignore_eovercrowded = true;
            if (sock->Write(&out, &wopt) != 0) {
                LOG_EVERY_SECOND(WARNING) << "Fail to write ordered responses into " << sock->description();
            }
        }
    }
}

}  // namespace mrpc
