#include "net/input_messenger.h"

#include <cerrno>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/fiber.h"
#include "rpc/errno.h"

DEFINE_bool(log_unknown_protocol, false, "log bytes of connections speaking no known protocol");

namespace mrpc {

static const size_t kMinOnceRead = 8192;  // one default block: a burst of small messages in one read
static const size_t kMaxOnceRead = 524288;

InputMessenger::InputMessenger(size_t capacity) : _capacity(capacity) {}
InputMessenger::~InputMessenger() {}

int InputMessenger::AddHandler(const InputMessageHandler& h) {
    if (!h.parse || !h.process) return -1;
    for (auto& x : _handlers) {
        if (x.parse == h.parse && x.process == h.process) return 0;  // dup
    }
    if (_handlers.size() >= _capacity) return -1;
    _handlers.push_back(h);
    return 0;
}

int InputMessenger::AddNonProtocolHandler(const InputMessageHandler& h) { return AddHandler(h); }

int InputMessenger::Create(const SocketOptions& options, SocketId* id) {
    SocketOptions opt = options;
    opt.user = this;
    opt.on_edge_triggered_events = OnNewMessages;
    return Socket::Create(opt, id);
}

ParseResult InputMessenger::CutInputMessage(Socket* m, size_t* index, bool read_eof) {
    const int preferred = m->_preferred_index;
    if (preferred >= 0 && (size_t)preferred < _handlers.size()) {
        const InputMessageHandler& h = _handlers[preferred];
        ParseResult r = h.parse(&m->_read_buf, m, read_eof, h.arg);
        if (r.is_ok() || r.error() == PARSE_ERROR_NOT_ENOUGH_DATA) {
            *index = (size_t)preferred;
            return r;
        }
        if (r.error() != PARSE_ERROR_TRY_OTHERS) return r;
    }
    for (size_t i = 0; i < _handlers.size(); ++i) {
        if ((int)i == preferred) continue;
        const InputMessageHandler& h = _handlers[i];
        ParseResult r = h.parse(&m->_read_buf, m, read_eof, h.arg);
        if (r.is_ok()) {
            m->_preferred_index = (int)i;
            *index = i;
            return r;
        }
        if (r.error() != PARSE_ERROR_TRY_OTHERS) {
            // a protocol that installed its parsing context owns the
            // connection even before its first complete message (the redis
            // server runs commands inside parse and always asks for more):
            // later reads go to it first, so a partial value at the front of
            // the buffer is never offered to the other protocols
            if (r.error() == PARSE_ERROR_NOT_ENOUGH_DATA && m->parsing_context() != nullptr) {
                m->_preferred_index = (int)i;
            }
            *index = i;
            return r;
        }
    }
    if (m->_read_buf.empty()) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    return MakeParseError(PARSE_ERROR_TRY_OTHERS);
}

static void* ProcessInputMessage(void* arg) {
    InputMessageBase* msg = static_cast<InputMessageBase*>(arg);
    msg->_process(msg);
    return nullptr;
}

void QueueOrProcessMessage(InputMessageBase* msg, bool in_place) {
    if (in_place) {
        ProcessInputMessage(msg);
        return;
    }
    fiber::fiber_t th;
    fiber::Attr attr(fiber::STACK_NORMAL, fiber::ATTR_NOSIGNAL);
    if (fiber::start_background(&th, &attr, ProcessInputMessage, msg) != 0) ProcessInputMessage(msg);
}

void InputMessenger::OnNewMessages(Socket* m) {
    InputMessenger* messenger = static_cast<InputMessenger*>(m->user());
    int progress = Socket::PROGRESS_INIT;
    InputMessageBase* last = nullptr;
    int num_queued = 0;
    bool read_eof = false;
    bool failed = false;
    while (!read_eof && !failed) {
        size_t once = (size_t)(m->_avg_msg_size * 16);
        if (once < kMinOnceRead) once = kMinOnceRead;
        if (once > kMaxOnceRead) once = kMaxOnceRead;
        const ssize_t nr = m->DoRead(once);
        if (nr <= 0) {
            if (nr == 0) {
                read_eof = true;
            } else if (errno == EAGAIN || errno == EWOULDBLOCK) {
                if (!m->MoreReadEvents(&progress)) break;
                continue;
            } else if (errno == EINTR) {
                continue;
            } else {
                m->SetFailed(errno, "fail to read from fd=%d: %s", m->fd(), ErrorText(errno));
                break;
            }
        }
        for (;;) {
            size_t index = 0;
            ParseResult pr = messenger->CutInputMessage(m, &index, read_eof);
            if (!pr.is_ok()) {
                if (pr.error() == PARSE_ERROR_NOT_ENOUGH_DATA) break;
                if (pr.error() == PARSE_ERROR_TRY_OTHERS) {
                    if (FLAGS_log_unknown_protocol) {
                        LOG(WARNING) << "Unknown protocol from " << m->remote_side() << ": "
                                     << m->_read_buf.to_string().substr(0, 64);
                    }
                    m->SetFailed(EREQUEST, "unknown protocol from %s", m->remote_side().to_string().c_str());
                } else {
                    m->SetFailed(EREQUEST, "fail to parse message from %s: %s", m->remote_side().to_string().c_str(),
                                 ParseErrorToString(pr.error()));
                }
                failed = true;
                break;
            }
            InputMessageBase* msg = pr.message();
            if (msg == nullptr) continue;  // consumed inside parse (ordered frames)
            const InputMessageHandler& h = messenger->_handlers[index];
            msg->_process = h.process;
            msg->_arg = h.arg;
            msg->_received_us = monotonic_us();
            m->AddRef();
            msg->_socket.reset(m);
            m->in_messages.fetch_add(1, std::memory_order_relaxed);
            if (h.verify && !m->_server_verified.load(std::memory_order_acquire)) {
                if (!h.verify(msg)) {
                    m->SetFailed(ERPCAUTH, "fail to authenticate %s", m->remote_side().to_string().c_str());
                    msg->Destroy();
                    failed = true;
                    break;
                }
                m->_server_verified.store(true, std::memory_order_release);
            }
            if (last) {
                QueueOrProcessMessage(last, false);
                ++num_queued;
            }
            last = msg;
        }
        // update average message size estimate
        if (nr > 0) {
            const int64_t avg = m->_avg_msg_size;
            m->_avg_msg_size = avg == 0 ? nr : (avg * 7 + nr) / 8;
        }
    }
    if (num_queued) fiber::flush();
    if (last) QueueOrProcessMessage(last, true);
    if (read_eof) m->SetFailed(EEOF, "got EOF of fd=%d", m->fd());
}

InputMessenger* get_client_side_messenger() {
    static InputMessenger* m = new InputMessenger;
    return m;
}

}  // namespace mrpc
