// Minimal in-tree declaration of the libibverbs ABI subset the ibverbs
// provider (rdma/provider.cc) uses, so the provider always compiles — there
// are no rdma-core headers in this build image or on the MI355X boxes.
//
// Layouts follow the stable libibverbs 1.1 ABI (IBVERBS_1.1 symbol version,
// the one `dlsym` resolves by default): the fields the provider touches sit
// at the same offsets as in rdma-core's <infiniband/verbs.h>, and structs
// the library writes into (ibv_port_attr, ibv_wc, ibv_qp_attr) are at least
// as large. The data-path calls (post_send/post_recv/poll_cq/
// req_notify_cq) are not exported symbols but function pointers in
// ibv_context::ops — exactly how the real header's static inlines reach
// them. A stub library implementing this ABI (tests/fake_ibverbs.cc) drives
// the provider in the unit tests; a real HCA is not available on this pool.
#pragma once

#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

namespace mrpc {
namespace rdma {
namespace verbs {

union ibv_gid {
    uint8_t raw[16];
    struct {
        uint64_t subnet_prefix;
        uint64_t interface_id;
    } global;
};

enum ibv_mtu { IBV_MTU_256 = 1, IBV_MTU_512 = 2, IBV_MTU_1024 = 3, IBV_MTU_2048 = 4, IBV_MTU_4096 = 5 };
enum ibv_port_state {
    IBV_PORT_NOP = 0,
    IBV_PORT_DOWN = 1,
    IBV_PORT_INIT = 2,
    IBV_PORT_ARMED = 3,
    IBV_PORT_ACTIVE = 4,
    IBV_PORT_ACTIVE_DEFER = 5
};

struct ibv_port_attr {
    ibv_port_state state;
    ibv_mtu max_mtu;
    ibv_mtu active_mtu;
    int gid_tbl_len;
    uint32_t port_cap_flags;
    uint32_t max_msg_sz;
    uint32_t bad_pkey_cntr;
    uint32_t qkey_viol_cntr;
    uint16_t pkey_tbl_len;
    uint16_t lid;
    uint16_t sm_lid;
    uint8_t lmc;
    uint8_t max_vl_num;
    uint8_t sm_sl;
    uint8_t subnet_timeout;
    uint8_t init_type_reply;
    uint8_t active_width;
    uint8_t active_speed;
    uint8_t phys_state;
    uint8_t link_layer;
    uint8_t flags;
    uint16_t port_cap_flags2;
    uint32_t active_speed_ex;
    uint8_t reserved_[32];  // room for later extensions written by the library
};

enum ibv_wc_status { IBV_WC_SUCCESS = 0 };
enum ibv_wc_opcode {
    IBV_WC_SEND = 0,
    IBV_WC_RDMA_WRITE = 1,
    IBV_WC_RDMA_READ = 2,
    IBV_WC_RECV = 1 << 7,
    IBV_WC_RECV_RDMA_WITH_IMM = (1 << 7) + 1
};
enum { IBV_WC_GRH = 1 << 0, IBV_WC_WITH_IMM = 1 << 1 };

struct ibv_wc {
    uint64_t wr_id;
    ibv_wc_status status;
    ibv_wc_opcode opcode;
    uint32_t vendor_err;
    uint32_t byte_len;
    uint32_t imm_data;  // network byte order
    uint32_t qp_num;
    uint32_t src_qp;
    unsigned int wc_flags;
    uint16_t pkey_index;
    uint16_t slid;
    uint8_t sl;
    uint8_t dlid_path_bits;
};

struct ibv_sge {
    uint64_t addr;
    uint32_t length;
    uint32_t lkey;
};

enum ibv_wr_opcode {
    IBV_WR_RDMA_WRITE = 0,
    IBV_WR_RDMA_WRITE_WITH_IMM = 1,
    IBV_WR_SEND = 2,
    IBV_WR_SEND_WITH_IMM = 3,
    IBV_WR_RDMA_READ = 4
};
enum { IBV_SEND_FENCE = 1, IBV_SEND_SIGNALED = 2, IBV_SEND_SOLICITED = 4, IBV_SEND_INLINE = 8 };

struct ibv_ah;
struct ibv_mw;
struct ibv_mr;

struct ibv_mw_bind_info {
    ibv_mr* mr;
    uint64_t addr;
    uint64_t length;
    unsigned int mw_access_flags;
};

struct ibv_send_wr {
    uint64_t wr_id;
    ibv_send_wr* next;
    ibv_sge* sg_list;
    int num_sge;
    ibv_wr_opcode opcode;
    unsigned int send_flags;
    uint32_t imm_data;  // network byte order
    union {
        struct {
            uint64_t remote_addr;
            uint32_t rkey;
        } rdma;
        struct {
            uint64_t remote_addr;
            uint64_t compare_add;
            uint64_t swap;
            uint32_t rkey;
        } atomic;
        struct {
            ibv_ah* ah;
            uint32_t remote_qpn;
            uint32_t remote_qkey;
        } ud;
    } wr;
    union {
        struct {
            uint32_t remote_srqn;
        } xrc;
    } qp_type;
    union {
        struct {
            ibv_mw* mw;
            uint32_t rkey;
            ibv_mw_bind_info bind_info;
        } bind_mw;
        struct {
            void* hdr;
            uint16_t hdr_sz;
            uint16_t mss;
        } tso;
    };
};

struct ibv_recv_wr {
    uint64_t wr_id;
    ibv_recv_wr* next;
    ibv_sge* sg_list;
    int num_sge;
};

struct ibv_device;
struct ibv_context;
struct ibv_cq;
struct ibv_qp;
struct ibv_srq;
struct ibv_pd;

// Data-path entry points live in the context's ops table; the other slots
// are compat placeholders the library fills and we never call.
struct ibv_context_ops {
    void* compat_query_device;
    void* compat_query_port;
    void* compat_alloc_pd;
    void* compat_dealloc_pd;
    void* compat_reg_mr;
    void* compat_rereg_mr;
    void* compat_dereg_mr;
    void* alloc_mw;
    void* bind_mw;
    void* dealloc_mw;
    void* compat_create_cq;
    int (*poll_cq)(ibv_cq* cq, int num_entries, ibv_wc* wc);
    int (*req_notify_cq)(ibv_cq* cq, int solicited_only);
    void* compat_cq_event;
    void* compat_resize_cq;
    void* compat_destroy_cq;
    void* compat_create_srq;
    void* compat_modify_srq;
    void* compat_query_srq;
    void* compat_destroy_srq;
    int (*post_srq_recv)(ibv_srq* srq, ibv_recv_wr* wr, ibv_recv_wr** bad);
    void* compat_create_qp;
    void* compat_query_qp;
    void* compat_modify_qp;
    void* compat_destroy_qp;
    int (*post_send)(ibv_qp* qp, ibv_send_wr* wr, ibv_send_wr** bad);
    int (*post_recv)(ibv_qp* qp, ibv_recv_wr* wr, ibv_recv_wr** bad);
    void* compat_create_ah;
    void* compat_destroy_ah;
    void* compat_attach_mcast;
    void* compat_detach_mcast;
    void* compat_async_event;
};

struct ibv_context {
    ibv_device* device;
    ibv_context_ops ops;
    int cmd_fd;
    int async_fd;
    int num_comp_vectors;
    pthread_mutex_t mutex;
    void* abi_compat;
};

struct ibv_comp_channel {
    ibv_context* context;
    int fd;
    int refcnt;
};

struct ibv_pd {
    ibv_context* context;
    uint32_t handle;
};

struct ibv_mr {
    ibv_context* context;
    ibv_pd* pd;
    void* addr;
    size_t length;
    uint32_t handle;
    uint32_t lkey;
    uint32_t rkey;
};

struct ibv_cq {
    ibv_context* context;
    ibv_comp_channel* channel;
    void* cq_context;
    uint32_t handle;
    int cqe;
    pthread_mutex_t mutex;
    pthread_cond_t cond;
    uint32_t comp_events_completed;
    uint32_t async_events_completed;
};

enum ibv_qp_state {
    IBV_QPS_RESET = 0,
    IBV_QPS_INIT = 1,
    IBV_QPS_RTR = 2,
    IBV_QPS_RTS = 3,
    IBV_QPS_SQD = 4,
    IBV_QPS_SQE = 5,
    IBV_QPS_ERR = 6
};
enum ibv_qp_type { IBV_QPT_RC = 2, IBV_QPT_UC = 3, IBV_QPT_UD = 4 };
enum ibv_mig_state { IBV_MIG_MIGRATED = 0, IBV_MIG_REARM = 1, IBV_MIG_ARMED = 2 };

struct ibv_qp {
    ibv_context* context;
    void* qp_context;
    ibv_pd* pd;
    ibv_cq* send_cq;
    ibv_cq* recv_cq;
    ibv_srq* srq;
    uint32_t handle;
    uint32_t qp_num;
    ibv_qp_state state;
    ibv_qp_type qp_type;
    pthread_mutex_t mutex;
    pthread_cond_t cond;
    uint32_t events_completed;
};

struct ibv_qp_cap {
    uint32_t max_send_wr;
    uint32_t max_recv_wr;
    uint32_t max_send_sge;
    uint32_t max_recv_sge;
    uint32_t max_inline_data;
};

struct ibv_qp_init_attr {
    void* qp_context;
    ibv_cq* send_cq;
    ibv_cq* recv_cq;
    ibv_srq* srq;
    ibv_qp_cap cap;
    ibv_qp_type qp_type;
    int sq_sig_all;
};

struct ibv_global_route {
    ibv_gid dgid;
    uint32_t flow_label;
    uint8_t sgid_index;
    uint8_t hop_limit;
    uint8_t traffic_class;
};

struct ibv_ah_attr {
    ibv_global_route grh;
    uint16_t dlid;
    uint8_t sl;
    uint8_t src_path_bits;
    uint8_t static_rate;
    uint8_t is_global;
    uint8_t port_num;
};

struct ibv_qp_attr {
    ibv_qp_state qp_state;
    ibv_qp_state cur_qp_state;
    ibv_mtu path_mtu;
    ibv_mig_state path_mig_state;
    uint32_t qkey;
    uint32_t rq_psn;
    uint32_t sq_psn;
    uint32_t dest_qp_num;
    unsigned int qp_access_flags;
    ibv_qp_cap cap;
    ibv_ah_attr ah_attr;
    ibv_ah_attr alt_ah_attr;
    uint16_t pkey_index;
    uint16_t alt_pkey_index;
    uint8_t en_sqd_async_notify;
    uint8_t sq_draining;
    uint8_t max_rd_atomic;
    uint8_t max_dest_rd_atomic;
    uint8_t min_rnr_timer;
    uint8_t port_num;
    uint8_t timeout;
    uint8_t retry_cnt;
    uint8_t rnr_retry;
    uint8_t alt_port_num;
    uint8_t alt_timeout;
    uint32_t rate_limit;
};

enum ibv_qp_attr_mask {
    IBV_QP_STATE = 1 << 0,
    IBV_QP_CUR_STATE = 1 << 1,
    IBV_QP_EN_SQD_ASYNC_NOTIFY = 1 << 2,
    IBV_QP_ACCESS_FLAGS = 1 << 3,
    IBV_QP_PKEY_INDEX = 1 << 4,
    IBV_QP_PORT = 1 << 5,
    IBV_QP_QKEY = 1 << 6,
    IBV_QP_AV = 1 << 7,
    IBV_QP_PATH_MTU = 1 << 8,
    IBV_QP_TIMEOUT = 1 << 9,
    IBV_QP_RETRY_CNT = 1 << 10,
    IBV_QP_RNR_RETRY = 1 << 11,
    IBV_QP_RQ_PSN = 1 << 12,
    IBV_QP_MAX_QP_RD_ATOMIC = 1 << 13,
    IBV_QP_ALT_PATH = 1 << 14,
    IBV_QP_MIN_RNR_TIMER = 1 << 15,
    IBV_QP_SQ_PSN = 1 << 16,
    IBV_QP_MAX_DEST_RD_ATOMIC = 1 << 17,
    IBV_QP_PATH_MIG_STATE = 1 << 18,
    IBV_QP_CAP = 1 << 19,
    IBV_QP_DEST_QPN = 1 << 20
};

enum ibv_access_flags {
    IBV_ACCESS_LOCAL_WRITE = 1,
    IBV_ACCESS_REMOTE_WRITE = 2,
    IBV_ACCESS_REMOTE_READ = 4,
    IBV_ACCESS_REMOTE_ATOMIC = 8
};

// Exported entry points (resolved with dlsym; signatures of IBVERBS_1.1).
using ibv_get_device_list_fn = ibv_device** (*)(int* num_devices);
using ibv_free_device_list_fn = void (*)(ibv_device** list);
using ibv_get_device_name_fn = const char* (*)(ibv_device* device);
using ibv_open_device_fn = ibv_context* (*)(ibv_device* device);
using ibv_close_device_fn = int (*)(ibv_context* context);
using ibv_alloc_pd_fn = ibv_pd* (*)(ibv_context* context);
using ibv_dealloc_pd_fn = int (*)(ibv_pd* pd);
using ibv_reg_mr_fn = ibv_mr* (*)(ibv_pd* pd, void* addr, size_t length, int access);
using ibv_reg_dmabuf_mr_fn = ibv_mr* (*)(ibv_pd* pd, uint64_t offset, size_t length, uint64_t iova, int fd,
                                         int access);
using ibv_dereg_mr_fn = int (*)(ibv_mr* mr);
using ibv_create_comp_channel_fn = ibv_comp_channel* (*)(ibv_context* context);
using ibv_destroy_comp_channel_fn = int (*)(ibv_comp_channel* channel);
using ibv_create_cq_fn = ibv_cq* (*)(ibv_context* context, int cqe, void* cq_context, ibv_comp_channel* channel,
                                     int comp_vector);
using ibv_destroy_cq_fn = int (*)(ibv_cq* cq);
using ibv_get_cq_event_fn = int (*)(ibv_comp_channel* channel, ibv_cq** cq, void** cq_context);
using ibv_ack_cq_events_fn = void (*)(ibv_cq* cq, unsigned int nevents);
using ibv_create_qp_fn = ibv_qp* (*)(ibv_pd* pd, ibv_qp_init_attr* attr);
using ibv_destroy_qp_fn = int (*)(ibv_qp* qp);
using ibv_modify_qp_fn = int (*)(ibv_qp* qp, ibv_qp_attr* attr, int attr_mask);
using ibv_query_port_fn = int (*)(ibv_context* context, uint8_t port_num, ibv_port_attr* attr);
using ibv_query_gid_fn = int (*)(ibv_context* context, uint8_t port_num, int index, ibv_gid* gid);

}  // namespace verbs
}  // namespace rdma
}  // namespace mrpc
