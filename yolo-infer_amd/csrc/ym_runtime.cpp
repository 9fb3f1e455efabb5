// yolomi runtime: model-blob parsing, device weight/workspace arena, per-op launch, HIP-graph cache, C-ABI.
//
// This is the native replacement for the Ultralytics predictor loop that `YOLO11Model.predict` delegates to
// (/root/reference/core/model.py:118-133): per batch it replays ONE captured HIP graph of the whole forward
// (input /255 rule → 80+ fused conv launches → attention → decode → NMS), so the Python host issues one call.
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/yolomi.h"
#include "ym_common.h"

namespace {

thread_local std::string g_err;

// YM_SEGV_TRACE=1: on SIGSEGV / SIGBUS print the native backtrace (library + offset per frame) to stderr, then hand
// the signal to the handler installed before ours (Python's faulthandler under pytest, which prints the Python
// stack), so a host crash inside the runtime leaves a trace that names the frame.
struct sigaction g_prev_sig[2];
void segv_trace(int sig, siginfo_t* si, void* uc) {
  static const char msg[] = "[yolomi] fatal signal, native backtrace:\n";
  void* fr[64];
  const int n = backtrace(fr, 64);
  if (write(2, msg, sizeof msg - 1) < 0) {}
  backtrace_symbols_fd(fr, n, 2);
  const struct sigaction& p = g_prev_sig[sig == SIGBUS];
  if ((p.sa_flags & SA_SIGINFO) && p.sa_sigaction) return p.sa_sigaction(sig, si, uc);
  if (!(p.sa_flags & SA_SIGINFO) && p.sa_handler != SIG_DFL && p.sa_handler != SIG_IGN) return p.sa_handler(sig);
  signal(sig, SIG_DFL);
  raise(sig);
}
__attribute__((constructor)) void install_segv_trace() {
  const char* e = getenv("YM_SEGV_TRACE");
  if (!e || !*e || *e == '0') return;
  void* warm[2];
  (void)backtrace(warm, 2);  // loads the unwinder now, not inside the handler
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = segv_trace;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_prev_sig[0]);
  sigaction(SIGBUS, &sa, &g_prev_sig[1]);
}

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCK(x)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) return fail(YM_EHIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

constexpr int32_t kMagic = 0x4C504D59;  // 'YMPL'
constexpr int kHdr = 32, kBufRec = 8, kOpRec = 32, kNameLen = 48;
constexpr int kSplitCounters = 16384;  // split-K tiles per conv launch (csrc/ym_conv_dma.hip)
constexpr int kChainCtl = 4096;
constexpr float kPresortConf = 0.1f;  // NMS keys presorted over several workgroups below this conf (ym_misc.hip)        // ready counters (+ done, give-up words) of the persistent chain kernel
constexpr int kMaxLanes = 4;           // concurrent batch slices in one forward graph (<= GPU_MAX_HW_QUEUES)
constexpr size_t kMaxGraphs = 16;      // captured forwards cached per context (the oldest is retired first)
constexpr size_t kMiscBytes = 16384;  // ym_ctx::d_misc

enum OpKind { OP_INPUT = 1, OP_CONV = 2, OP_DW = 3, OP_SPPF = 4, OP_ATTN = 5, OP_DECODE = 6, OP_NMS = 7, OP_REQ = 8 };

struct BufDesc {
  int C, f, f32;
};

struct Op {
  int32_t r[kOpRec];
  char name[kNameLen];
};

struct GraphKey {
  int B, H, W;
  const void* in;
  const void* dets;
  const void* counts;
  const void* stream_unused;
  ym_infer_args args;
  bool operator==(const GraphKey& o) const { return memcmp(this, &o, sizeof(GraphKey)) == 0; }
};

// A captured forward.  The detection rows are the caller's (a fresh tensor per predict() call, so the Results of
// earlier calls stay valid without a copy): the key leaves `dets` out when the graph's NMS nodes were found, and a
// replay for other rows re-points those nodes (hipGraphExecKernelNodeSetParams; the lanes' row offsets kept).
struct GraphEntry {
  GraphKey key;
  hipGraph_t graph;
  hipGraphExec_t exec;
  float* dets = nullptr;                 // the rows the exec's NMS nodes write now
  hipEvent_t done = nullptr;             // recorded behind every launch of `exec` (retire_graph waits on it)
  std::vector<hipGraphNode_t> nms_nodes;  // empty: dets is part of the key
  std::vector<NmsArgs> nms_args;
};

// The NMS kernel nodes of a captured forward and their arguments (false when none is found: the caller keys the
// graph on the output pointer instead)
bool find_nms_nodes(GraphEntry& ge) {
  size_t nn = 0;
  if (hipGraphGetNodes(ge.graph, nullptr, &nn) != hipSuccess || nn == 0) return false;
  std::vector<hipGraphNode_t> nodes(nn);
  if (hipGraphGetNodes(ge.graph, nodes.data(), &nn) != hipSuccess) return false;
  for (hipGraphNode_t n : nodes) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(n, &t) != hipSuccess || t != hipGraphNodeTypeKernel) continue;
    hipKernelNodeParams p{};
    if (hipGraphKernelNodeGetParams(n, &p) != hipSuccess || p.func != ym_nms_kernel()) continue;
    if (!p.kernelParams || !p.kernelParams[0]) return false;
    ge.nms_nodes.push_back(n);
    ge.nms_args.push_back(*static_cast<const NmsArgs*>(p.kernelParams[0]));
  }
  if (ge.nms_nodes.empty()) return false;
  for (const NmsArgs& a : ge.nms_args)  // every node writes inside the captured rows
    if (a.dets < ge.dets) {
      ge.nms_nodes.clear();
      ge.nms_args.clear();
      return false;
    }
  return true;
}

int repoint_dets(GraphEntry& ge, float* d_dets) {
  for (size_t j = 0; j < ge.nms_nodes.size(); ++j) {
    NmsArgs na = ge.nms_args[j];
    na.dets = d_dets + (na.dets - ge.dets);
    if (na.counts2)  // the counts behind the rows move with them
      na.counts2 = reinterpret_cast<int*>(reinterpret_cast<char*>(na.counts2) +
                                          (reinterpret_cast<char*>(d_dets) - reinterpret_cast<char*>(ge.dets)));
    hipKernelNodeParams p{};
    HIPCK(hipGraphKernelNodeGetParams(ge.nms_nodes[j], &p));
    void* args[] = {&na};
    p.kernelParams = args;
    p.extra = nullptr;
    HIPCK(hipGraphExecKernelNodeSetParams(ge.exec, ge.nms_nodes[j], &p));
    ge.nms_args[j] = na;
  }
  ge.dets = d_dets;
  return YM_OK;
}

// Destroy a captured forward only after its last launch has finished on whatever stream it was replayed on: the
// HIP runtime may still hold the exec's launch state (kernel arguments, the packet chain) while it is in flight.
void retire_graph(GraphEntry& g) {
  if (g.done) {
    (void)hipEventSynchronize(g.done);
    (void)hipEventDestroy(g.done);
    g.done = nullptr;
  }
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  if (g.graph) (void)hipGraphDestroy(g.graph);
  g.exec = nullptr;
  g.graph = nullptr;
}

}  // namespace

struct ym_ctx {
  int device = 0;
  ym_model_desc desc{};
  bool loaded = false;
  // plan
  int dtype = YM_DT_F16, task = 0, nc = 80, nm = 0, reg_max = 16, nl = 3;
  int strides[4] = {8, 16, 32, 0};
  int input_buf = -1, anchor_buf = -1, proto_buf = -1, no = 0;
  float* d_lowres = nullptr;  // Segment mask assembly scratch (ym_masks)
  char* d_misc = nullptr;     // 16 KB: ym_input_max statistics region, ym_broadcast_weights control words
  size_t lowres_bytes = 0;
  std::vector<BufDesc> bufs;
  std::vector<Op> ops;
  char* d_weights = nullptr;
  std::vector<char> blob_host;  // the loaded blob as received (what ym_broadcast_weights sends from the root)
  size_t off_wstem = 0;  // stem weights re-laid out as fp32 [27][N] behind the blob's weights (ym_stem.hip)
  size_t off_wtap0 = 0;            // int8 plans: the 3x3 convs' [9][N] int32 tap sums, behind the stem weights
  std::vector<size_t> off_wtap;    // per op: 1 + byte offset from off_wtap0 (0: none)
  // branch schedule of a one-lane forward (ops of independent DAG branches on up to kMaxLanes streams)
  int nbr = 1;
  std::vector<int> br_of;                // per op: branch stream
  std::vector<std::vector<int>> br_wait; // per op: earlier ops (other streams) whose events it waits for
  std::vector<char> br_rec;              // per op: record its event after it
  std::vector<hipEvent_t> op_ev;
  size_t wbytes = 0;
  // workspace for the current (B, H, W)
  int cB = 0, cH = 0, cW = 0;
  char* d_arena = nullptr;
  size_t arena_bytes = 0;
  std::vector<size_t> buf_off;
  size_t off_boxes = 0, off_scores = 0, off_cls = 0, off_keys = 0, off_keys2 = 0, off_counts = 0, off_ctl = 0, off_sboxes = 0,
         off_sareas = 0, off_sup = 0, off_slab = 0, off_cnt = 0, off_chain = 0, slab_bytes = 0;
  int A = 0, kstride = 0;
  int lvl_W[4] = {0}, lvl_off[4] = {0};
  hipStream_t cap_stream = nullptr;
  // lanes: the batch is cut into image slices whose op chains are captured as parallel branches of one graph, so
  // the fixed per-launch latency of one slice's small kernels overlaps the other slices' work
  hipStream_t lane_streams[kMaxLanes] = {};
  hipEvent_t fork_ev = nullptr, join_ev[kMaxLanes] = {};
  int lane = 0, lane_img0 = 0;  // lane / first image of the ops being launched
  int call_B = 0;               // images of the forward being launched (all lanes)
  std::vector<GraphEntry> graphs;
  // the previous forward: every forward of a context uses the same arena, NMS scratch, split-K slabs /
  // counters and input_stats ticket, so a forward launched on another stream than the previous one first waits for
  // it (ym_infer: hipStreamWaitEvent); last_ev is the replayed graph's `done` event or fwd_ev (eager forwards)
  hipStream_t last_st = nullptr;
  hipEvent_t last_ev = nullptr, fwd_ev = nullptr;
  int order_after_last(hipStream_t st) {
    if (last_ev && last_st != st) {
      const hipError_t e = hipStreamWaitEvent(st, last_ev, 0);
      if (e != hipSuccess) return fail(YM_EHIP, "stream order: %s", hipGetErrorString(e));
    }
    return YM_OK;
  }
  void retire(GraphEntry& g) {  // retire_graph, forgetting last_ev when it is that graph's event (now complete)
    if (g.done && g.done == last_ev) last_ev = nullptr;
    retire_graph(g);
  }
  std::vector<hipEvent_t> prof_events;
  float* const* calib_raw = nullptr;  // ym_calibrate: per-op pre-activation output buffers (f32 plans)
  // per-shape, per-op conv tile configuration (-1 = heuristic); set by ym_tune / ym_set_op_cfg
  struct ShapeCfg {
    int B, H, W;
    std::vector<int> cfg;
  };
  std::vector<ShapeCfg> cfgs;
  const std::vector<int>* find_cfg(int B, int H, int W) const {
    for (const auto& e : cfgs)
      if (e.B == B && e.H == H && e.W == W) return &e.cfg;
    return nullptr;
  }
  void put_cfg(int B, int H, int W, std::vector<int> v) {
    for (auto& e : cfgs)
      if (e.B == B && e.H == H && e.W == W) { e.cfg = std::move(v); return; }
    cfgs.push_back({B, H, W, std::move(v)});
  }
  void drop_cfg(int B, int H, int W) {
    for (size_t i = 0; i < cfgs.size(); ++i)
      if (cfgs[i].B == B && cfgs[i].H == H && cfgs[i].W == W) { cfgs.erase(cfgs.begin() + i); return; }
  }
  int op_cfg(long i, int B) const {  // for the current workspace height/width
    const std::vector<int>* v = find_cfg(B, cH, cW);
    return (v && i >= 0 && i < (long)v->size()) ? (*v)[i] : -1;
  }

  ~ym_ctx() {
    (void)hipSetDevice(device);
    clear_graphs();
    for (auto e : prof_events) (void)hipEventDestroy(e);
    if (d_arena) (void)hipFree(d_arena);
    if (d_weights) (void)hipFree(d_weights);
    if (d_lowres) (void)hipFree(d_lowres);
    if (d_misc) (void)hipFree(d_misc);
    if (cap_stream) (void)hipStreamDestroy(cap_stream);
    for (int l = 0; l < kMaxLanes; ++l) {
      if (lane_streams[l]) (void)hipStreamDestroy(lane_streams[l]);
      if (join_ev[l]) (void)hipEventDestroy(join_ev[l]);
    }
    if (fork_ev) (void)hipEventDestroy(fork_ev);
    if (fwd_ev) (void)hipEventDestroy(fwd_ev);
    for (hipEvent_t e : op_ev) (void)hipEventDestroy(e);
  }
  void clear_graphs() {
    for (auto& g : graphs) retire(g);
    graphs.clear();
  }
  int buf_P(int b) const {
    const BufDesc& d = bufs[b];
    if (d.f == 0) return A;
    return (cH / d.f) * (cW / d.f);
  }
  int buf_H(int b) const { return bufs[b].f == 0 ? 1 : cH / bufs[b].f; }
  int buf_Wd(int b) const { return bufs[b].f == 0 ? A : cW / bufs[b].f; }
  int elem(int b) const { return (bufs[b].f32 || ym_dt_f32s(dtype)) ? 4 : (ym_dt_q8(dtype) ? 1 : 2); }
  template <typename T> const T* wptr(int32_t off) const {
    return reinterpret_cast<const T*>(d_weights + (size_t)(uint32_t)off);
  }
  float* raw_of(const Op& op) const { return calib_raw ? calib_raw[&op - ops.data()] : nullptr; }
  // buffer b of the current lane: its image slice of the whole-batch buffer (all buffers are image-major)
  void* bptr(int b) const {
    return d_arena + buf_off[b] + (size_t)lane_img0 * buf_P(b) * bufs[b].C * elem(b);
  }
  template <typename T> T* scratch(size_t off, size_t per_image_bytes) const {
    return reinterpret_cast<T*>(d_arena + off + (size_t)lane_img0 * per_image_bytes);
  }
};

namespace {

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

int ensure_workspace(ym_ctx* c, int B, int H, int W) {
  if (c->d_arena && B <= c->cB && H == c->cH && W == c->cW) return YM_OK;
  const int nB = (H == c->cH && W == c->cW && B < c->cB) ? c->cB : B;
  c->clear_graphs();
  if (c->d_arena) {
    HIPCK(hipDeviceSynchronize());  // eager forwards on any stream may still read or write the old arena
    HIPCK(hipFree(c->d_arena));
    c->d_arena = nullptr;
  }
  c->cB = nB;
  c->cH = H;
  c->cW = W;
  c->A = 0;
  for (int l = 0; l < c->nl; ++l) {
    c->lvl_off[l] = c->A;
    c->lvl_W[l] = W / c->strides[l];
    c->A += (H / c->strides[l]) * (W / c->strides[l]);
  }
  c->kstride = 1;
  while (c->kstride < c->A) c->kstride <<= 1;
  size_t off = 0;
  c->buf_off.assign(c->bufs.size(), 0);
  for (size_t b = 0; b < c->bufs.size(); ++b) {
    c->buf_off[b] = off;
    if ((int)b == c->input_buf) continue;  // the stem conv reads the caller's NCHW fp32 batch directly
    off = align_up(off + (size_t)nB * c->buf_P((int)b) * c->bufs[b].C * c->elem((int)b), 256);
  }
  const size_t BA = (size_t)nB * c->A;
  c->off_boxes = off;  off = align_up(off + BA * 16, 256);
  c->off_scores = off; off = align_up(off + BA * 4, 256);
  c->off_cls = off;    off = align_up(off + BA * 4, 256);
  c->off_keys = off;   off = align_up(off + (size_t)nB * c->kstride * 8, 256);
  c->off_keys2 = off;  off = align_up(off + (size_t)nB * c->kstride * 8, 256);  // NMS presort chunks
  c->off_counts = off; off = align_up(off + (size_t)nB * 4, 256);
  c->off_ctl = off;    off = align_up(off + YM_CTL_BYTES, 256);
  c->off_sboxes = off; off = align_up(off + BA * 16, 256);
  c->off_sareas = off; off = align_up(off + BA * 4, 256);
  c->off_sup = off;    off = align_up(off + BA, 256);
  // split-K workspace of the LDS-DMA conv kernels: fp32 partial tiles + per-tile arrival counters
  c->slab_bytes = std::min<size_t>(std::max<size_t>(32u << 20, (size_t)nB << 22), 1u << 30);
  c->off_slab = off;   off = align_up(off + kMaxLanes * c->slab_bytes, 256);  // one slab region per lane
  c->off_cnt = off;    off = align_up(off + (size_t)kMaxLanes * kSplitCounters * 4, 256);
  c->off_chain = off;  off = align_up(off + (size_t)kChainCtl * 4, 256);  // persistent chain kernel's counters
  c->arena_bytes = off;
  hipError_t e = hipMalloc(&c->d_arena, off);
  if (e != hipSuccess) {
    c->d_arena = nullptr;
    c->cB = 0;
    return fail(YM_ENOMEM, "workspace hipMalloc(%zu) failed: %s", off, hipGetErrorString(e));
  }
  HIPCK(hipMemset(c->d_arena, 0, off));
  return YM_OK;
}

// Kernel arguments of a conv op for batch B at the current workspace shape.
int conv_args(ym_ctx* c, const Op& op, int B, const float* d_in, float in_eps, ConvArgs& a, int& out_f32) {
      const int32_t* r = op.r;
      a = ConvArgs{};
      a.wsc = a.wsc2 = 1.0f;
      const int pst = ym_debug_get(YM_DBG_PAIRST);  // (value + 1; 0: the default family mask 21)
      a.pst = pst ? pst - 1 : 21;
      const int k = r[1], s = r[2], cin = r[3], cout = r[4];
      const int b0 = r[6], b1 = r[10], bd = r[13], br = r[17];
      const int up0 = r[9];
      a.src0 = c->bptr(b0); a.s0_ctot = c->bufs[b0].C; a.s0_coff = r[7]; a.C0 = r[8];
      if (b0 == c->input_buf) {  // stem: NCHW fp32 source, LoadTensor /255 decided on device from ctl[0]
        a.src0 = nullptr;
        a.nchw = d_in;
        a.ctl = reinterpret_cast<const float*>(c->d_arena + c->off_ctl);
        a.eps = in_eps;
        a.wstem = reinterpret_cast<const float*>(c->d_weights + c->off_wstem);
      }
      a.s0_W = c->buf_Wd(b0); a.s0_P = c->buf_P(b0); a.up0 = up0;
      a.Hin = c->buf_H(b0) * (up0 ? 2 : 1);
      a.Win = c->buf_Wd(b0) * (up0 ? 2 : 1);
      if (b1 >= 0) {
        a.src1 = c->bptr(b1); a.s1_ctot = c->bufs[b1].C; a.s1_coff = r[11]; a.C1 = r[12]; a.s1_P = c->buf_P(b1);
        if (c->buf_H(b1) != a.Hin || c->buf_Wd(b1) != a.Win)
          return fail(YM_EBLOB, "op %s: concat sources disagree in shape", op.name);
      }
      a.k = k; a.s = s; a.pad = k / 2;
      a.Ho = (a.Hin + 2 * a.pad - k) / s + 1;
      a.Wo = (a.Win + 2 * a.pad - k) / s + 1;
      if (cin % 8 || (a.C0 + a.C1) != cin) return fail(YM_EBLOB, "op %s: cin %d not a multiple of 8", op.name, cin);
      a.Cin8 = cin / 8;
      if (ym_dt_q8(c->dtype)) {  // int8 / fp8 plans: K chunks of 16 channels (the stem keeps its 8-padded taps)
        if (b0 != c->input_buf) {
          if (cin % 16) return fail(YM_EBLOB, "op %s: int8 cin %d not a multiple of 16", op.name, cin);
          a.Cin8 = cin / 16;
        }
        a.q = c->wptr<QRec>(r[22]);
        a.sasw = c->wptr<float>(r[23]);
        a.biasi = c->wptr<int>(r[24]);
        const size_t oi = (size_t)(&op - c->ops.data());
        if (oi < c->off_wtap.size() && c->off_wtap[oi])
          a.wtap = reinterpret_cast<const int*>(c->d_weights + c->off_wtap0 + (c->off_wtap[oi] - 1));
      }
      if (c->dtype == YM_DT_X3 && b0 != c->input_buf) {  // pair layout: fp16 storage chunks per tap double
        a.x3 = 1;
        a.Cin8 = 2 * (cin / 8);
        // the packed weights are W·2^s (and W2·2^s2): yolomi/plan.py, record slots 22 / 23 (int8 plans only otherwise)
        if (r[22] < -64 || r[22] > 64 || r[23] < -64 || r[23] > 64)
          return fail(YM_EBLOB, "op %s: bad x3 weight scale exponents %d / %d", op.name, r[22], r[23]);
        a.wsc = ldexpf(1.0f, -r[22]);
        a.wsc2 = ldexpf(1.0f, -r[23]);
      }
      a.Kc = k * k * a.Cin8;
      a.Kpad = r[21];
      a.N = cout;
      a.w = c->d_weights + (size_t)(uint32_t)r[19];
      a.bias = reinterpret_cast<const float*>(c->d_weights + (size_t)(uint32_t)r[20]);
      a.act = r[5];
      if (r[30]) {  // fused pair (yolomi/arch.py fuse_pairs): a following 1x1 conv, output in dst/res
        if (c->dtype != YM_DT_F16 && c->dtype != YM_DT_X3)
          return fail(YM_EBLOB, "op %s: fused conv pairs are f16 / x3 only", op.name);
        a.w2 = c->d_weights + (size_t)(uint32_t)r[25];
        a.bias2 = reinterpret_cast<const float*>(c->d_weights + (size_t)(uint32_t)r[26]);
        a.N2 = r[27]; a.act2 = r[28]; a.Kpad2 = r[29]; a.k2 = r[30];
        if ((a.k2 != 1 && a.k2 != 3) || a.N2 <= 0 || a.Kpad2 < a.k2 * a.k2 * cout * (a.x3 ? 2 : 1) || r[31] < 0 || r[31] >= (int)c->bufs.size() || cout % 8 ||
            c->buf_H(r[31]) != a.Ho || c->buf_Wd(r[31]) != a.Wo || c->bufs[r[31]].C != cout || c->bufs[r[31]].f32)
          return fail(YM_EBLOB, "op %s: bad fused-pair geometry", op.name);
        if (ym_conv_num_cfgs_dt(c->dtype) > 255) return fail(YM_EBLOB, "split cfg encoding needs < 256 conv configs");
      }
      if (r[24] > 0 && !ym_dt_q8(c->dtype)) {  // fused depthwise (yolomi/arch.py fuse_dw): 1 + offset of [9][C] ‖ [C]
        if ((c->dtype != YM_DT_F16 && c->dtype != YM_DT_X3) || k != 1 || s != 1 || b1 >= 0 || up0 || r[30])
          return fail(YM_EBLOB, "op %s: a fused depthwise needs a single-source 1x1 conv of an f16 / x3 plan", op.name);
        a.dw_w = reinterpret_cast<const float*>(c->d_weights + (size_t)(uint32_t)(r[24] - 1));
        a.dw_b = a.dw_w + 9 * (size_t)cin;
        a.dw_act = 1;
      }
      a.shuffle = r[16];
      a.npr = a.shuffle ? cout / 4 : cout;
      a.dst = c->bptr(bd); a.d_ctot = c->bufs[bd].C; a.d_coff = r[14]; a.d_P = c->buf_P(bd);
      const int lvl = r[15];
      if (lvl >= 0) {
        a.d_pixoff = c->lvl_off[lvl];
        a.d_W = a.Wo;
        if (a.Wo != c->lvl_W[lvl]) return fail(YM_EBLOB, "op %s: head level width mismatch", op.name);
      } else {
        a.d_pixoff = 0;
        a.d_W = c->buf_Wd(bd);
        const int expect = a.shuffle ? 2 : 1;
        if (c->buf_H(bd) != expect * a.Ho || c->buf_Wd(bd) != expect * a.Wo)
          return fail(YM_EBLOB, "op %s: output %dx%d does not match dst buffer %dx%d", op.name, a.Ho, a.Wo,
                      c->buf_H(bd), c->buf_Wd(bd));
      }
      if (br >= 0) { a.res = c->bptr(br); a.r_ctot = c->bufs[br].C; a.r_coff = r[18]; a.r_P = c->buf_P(br); }
      a.M = B * a.Ho * a.Wo;
      a.fd_hw = ym_fdiv(a.Ho * a.Wo);
      a.fd_w = ym_fdiv(a.Wo);
      out_f32 = c->bufs[bd].f32 && c->dtype != YM_DT_F32;  // (x3: fp32 head rows, pair-layout activations)
      a.raw = c->raw_of(op);
      // operand extents in storage elements (the LDS-DMA buffer descriptors): fp16 halves of the x3 pairs
      const long xs = a.x3 ? 2 : 1;
      a.s0_elems = (b0 == c->input_buf) ? 0 : xs * c->cB * c->buf_P(b0) * c->bufs[b0].C;
      a.s1_elems = b1 >= 0 ? xs * c->cB * c->buf_P(b1) * c->bufs[b1].C : 0;
      a.slab = reinterpret_cast<float*>(c->d_arena + c->off_slab + (size_t)c->lane * c->slab_bytes);
      a.slab_cap = (long)c->slab_bytes;
      a.cnt = reinterpret_cast<int*>(c->d_arena + c->off_cnt) + (size_t)c->lane * kSplitCounters;
      a.cnt_cap = kSplitCounters;
      static const int pf_max = [] { const char* e = getenv("YM_DMA_PF"); return e ? atoi(e) : 0; }();
      a.pf = a.M <= pf_max;
      return YM_OK;
}

// A fused pair (ConvArgs::w2) run as its two convs: A writes the intermediate buffer (record r[31]), B reads it.
// The tuner picks this when the two tuned single launches beat every fused variant (op cfg kSplitTag + ...).
constexpr int kSplitTag = 1 << 20;  // op cfg = kSplitTag + 256 * cfg(A) + cfg(B)
void split_args(ym_ctx* c, const Op& op, const ConvArgs& a, ConvArgs& A, ConvArgs& Bc) {
  const int mid = op.r[31];
  A = a;
  A.w2 = nullptr; A.bias2 = nullptr; A.res = nullptr;
  A.dst = c->bptr(mid); A.d_ctot = c->bufs[mid].C; A.d_coff = 0; A.d_P = c->buf_P(mid); A.d_pixoff = 0;
  A.d_W = c->buf_Wd(mid);
  Bc = a;
  Bc.w2 = nullptr; Bc.bias2 = nullptr;
  Bc.src0 = c->bptr(mid); Bc.s0_ctot = c->bufs[mid].C; Bc.s0_coff = 0; Bc.C0 = a.N; Bc.s0_W = c->buf_Wd(mid);
  Bc.s0_P = c->buf_P(mid); Bc.up0 = 0;
  Bc.src1 = nullptr; Bc.C1 = 0; Bc.s1_elems = 0;
  Bc.Hin = a.Ho; Bc.Win = a.Wo; Bc.k = a.k2; Bc.s = 1; Bc.pad = a.k2 / 2;
  const int xs = a.x3 ? 2 : 1;  // x3: fp16 storage chunks of the pair layout
  Bc.Cin8 = xs * a.N / 8; Bc.Kc = a.k2 * a.k2 * Bc.Cin8; Bc.Kpad = a.Kpad2; Bc.N = a.N2; Bc.npr = a.N2;
  Bc.w = a.w2; Bc.bias = a.bias2; Bc.act = a.act2; Bc.wsc = a.wsc2;
  Bc.s0_elems = (long)xs * c->cB * c->buf_P(mid) * c->bufs[mid].C;
}

hipError_t launch_fused(ym_ctx* c, const Op& op, const ConvArgs& a, int out_f32, int cfg, hipStream_t st) {
  if (cfg < kSplitTag) {
    const hipError_t e = ym_launch_conv(c->dtype, out_f32, a, cfg, st);
    if (e != hipErrorInvalidValue) return e;
    cfg = kSplitTag + 256 * 255 + 255;  // no fused kernel takes this shape (e.g. a map width the Bottleneck kernel
  }                                     // does not tile): the two convs with their heuristic tiles
  ConvArgs A, Bc;
  split_args(c, op, a, A, Bc);
  const hipError_t e = ym_launch_conv(c->dtype, 0, A, ((cfg - kSplitTag) >> 8) & 255, st);
  return e != hipSuccess ? e : ym_launch_conv(c->dtype, out_f32, Bc, (cfg - kSplitTag) & 255, st);
}

int launch_op(ym_ctx* c, const Op& op, int B, const float* d_in, const ym_infer_args* args, float* d_dets,
              int* d_counts, hipStream_t st) {
  const int32_t* r = op.r;
  const int dt = c->dtype;
  hipError_t e = hipSuccess;
  switch (r[0]) {
    case OP_INPUT: {
      PrepArgs a{};
      a.in = d_in;
      a.out = c->bptr(c->input_buf);
      a.ctl = reinterpret_cast<float*>(c->d_arena + c->off_ctl);
      a.B = B; a.C = 3; a.H = c->cH; a.W = c->cW;
      a.eps = args->in_eps;
      a.batch_max = args->d_batch_max;
      a.cnt = reinterpret_cast<int*>(c->d_arena + c->off_cnt);
      a.cnt_len = kMaxLanes * kSplitCounters;
      e = ym_launch_prep(dt, a, reinterpret_cast<int*>(c->d_arena + c->off_counts), B, st);
      break;
    }
    case OP_CONV: {
      ConvArgs a{};
      int out_f32 = 0;
      const int rc = conv_args(c, op, B, d_in, args->in_eps, a, out_f32);
      if (rc) return rc;
      const int cfg = c->op_cfg(&op - c->ops.data(), B);
      e = a.nchw ? ym_launch_stem(dt, a, st)
                 : (a.w2 ? launch_fused(c, op, a, out_f32, cfg, st) : ym_launch_conv(dt, out_f32, a, cfg, st));
      break;
    }
    case OP_DW: {
      DwArgs a{};
      const int bs = r[6], bd = r[13];
      a.src = c->bptr(bs); a.s_ctot = c->bufs[bs].C; a.s_coff = r[7]; a.s_P = c->buf_P(bs);
      a.dst = c->bptr(bd); a.d_ctot = c->bufs[bd].C; a.d_coff = r[14]; a.d_P = c->buf_P(bd);
      a.w = reinterpret_cast<const float*>(c->d_weights + (size_t)(uint32_t)r[19]);
      a.bias = reinterpret_cast<const float*>(c->d_weights + (size_t)(uint32_t)r[20]);
      a.C = r[3]; a.act = r[5]; a.H = c->buf_H(bs); a.W = c->buf_Wd(bs); a.B = B;
      if (ym_dt_q8(dt)) {
        a.w = nullptr;
        a.wq = c->wptr<i8>(r[19]);
        a.q = c->wptr<QRec>(r[22]);
        a.sasw = c->wptr<float>(r[23]);
      }
      a.raw = c->raw_of(op);
      e = ym_launch_dwconv(dt, a, st);
      break;
    }
    case OP_SPPF: {
      PoolArgs a{};
      const int bb = r[13];
      a.buf = c->bptr(bb); a.ctot = c->bufs[bb].C; a.coff = r[7]; a.P = c->buf_P(bb);
      a.C = r[3]; a.H = c->buf_H(bb); a.W = c->buf_Wd(bb); a.B = B;
      e = ym_launch_sppf(dt, a, st);
      break;
    }
    case OP_ATTN: {
      AttnArgs a{};
      const int bq = r[6], bd = r[13];
      a.qkv = c->bptr(bq); a.q_ctot = c->bufs[bq].C; a.q_coff = r[7]; a.q_P = c->buf_P(bq);
      a.dst = c->bptr(bd); a.d_ctot = c->bufs[bd].C; a.d_coff = r[14]; a.d_P = c->buf_P(bd);
      a.pe_w = reinterpret_cast<const float*>(c->d_weights + (size_t)(uint32_t)r[19]);
      a.pe_b = reinterpret_cast<const float*>(c->d_weights + (size_t)(uint32_t)r[20]);
      a.C = r[3]; a.nh = r[4]; a.kd = r[5]; a.hd = r[9];
      a.H = c->buf_H(bq); a.W = c->buf_Wd(bq); a.N = a.H * a.W; a.B = B;
      memcpy(&a.scale, &r[21], 4);
      if (ym_dt_q8(dt)) {
        a.pe_w = nullptr;
        a.pe_wq = c->wptr<i8>(r[19]);
        a.q = c->wptr<QRec>(r[22]);
        a.pe_sasw = c->wptr<float>(r[23]);
      }
      a.raw = c->raw_of(op);
      e = ym_launch_attn(dt, a, st);
      break;
    }
    case OP_REQ: {
      if (!ym_dt_q8(dt)) return fail(YM_EBLOB, "op %s: requant in a non-quantized plan", op.name);
      ReqArgs a{};
      const int bs = r[6], bd = r[13];
      a.src = static_cast<const i8*>(c->bptr(bs)); a.s_ctot = c->bufs[bs].C; a.s_coff = r[7]; a.s_P = c->buf_P(bs);
      a.s_W = c->buf_Wd(bs); a.up = r[9];
      a.dst = static_cast<i8*>(c->bptr(bd)); a.d_ctot = c->bufs[bd].C; a.d_coff = r[14]; a.d_P = c->buf_P(bd);
      a.d_W = c->buf_Wd(bd);
      a.C = r[3]; a.H = c->buf_H(bd); a.W = c->buf_Wd(bd); a.B = B;
      if (c->buf_H(bs) * (a.up ? 2 : 1) != a.H || a.s_W * (a.up ? 2 : 1) != a.W)
        return fail(YM_EBLOB, "op %s: requant source/destination shapes disagree", op.name);
      a.q = c->wptr<QRec>(r[22]);
      e = ym_launch_requant(a, st, dt == YM_DT_F8);
      break;
    }
    case OP_DECODE: {
      DecodeArgs a{};
      a.anchors = reinterpret_cast<const float*>(c->bptr(c->anchor_buf));
      a.no_tot = c->bufs[c->anchor_buf].C;
      a.boxes = c->scratch<float4>(c->off_boxes, (size_t)c->A * 16);
      a.scores = c->scratch<float>(c->off_scores, (size_t)c->A * 4);
      a.cls = c->scratch<int>(c->off_cls, (size_t)c->A * 4);
      a.keys = c->scratch<unsigned long long>(c->off_keys, (size_t)c->kstride * 8);
      a.counts = c->scratch<int>(c->off_counts, 4);
      a.A = c->A; a.kstride = c->kstride; a.nc = c->nc; a.reg_max = c->reg_max; a.B = B; a.nl = c->nl;
      for (int l = 0; l < c->nl; ++l) {
        a.lvl_W[l] = c->lvl_W[l]; a.lvl_off[l] = c->lvl_off[l]; a.lvl_stride[l] = (float)c->strides[l];
      }
      a.conf = args->conf;
      a.has_classes = args->has_classes;
      for (int i = 0; i < 4; ++i) a.classes[i] = args->classes[i];
      e = ym_launch_decode(a, st);
      break;
    }
    case OP_NMS: {
      NmsArgs a{};
      a.anchors = reinterpret_cast<const float*>(c->bptr(c->anchor_buf));
      a.no_tot = c->bufs[c->anchor_buf].C;
      a.mask_off = c->no;
      a.boxes = c->scratch<const float4>(c->off_boxes, (size_t)c->A * 16);
      a.scores = c->scratch<const float>(c->off_scores, (size_t)c->A * 4);
      a.cls = c->scratch<const int>(c->off_cls, (size_t)c->A * 4);
      a.keys = c->scratch<unsigned long long>(c->off_keys, (size_t)c->kstride * 8);
      a.counts = c->scratch<const int>(c->off_counts, 4);
      a.sboxes = c->scratch<float4>(c->off_sboxes, (size_t)c->A * 16);
      a.sareas = c->scratch<float>(c->off_sareas, (size_t)c->A * 4);
      a.sup = c->scratch<unsigned char>(c->off_sup, (size_t)c->A);
      a.dets = d_dets;
      a.out_counts = d_counts;
      // counts_after_dets: this lane's images' words behind the WHOLE batch's rows (lane_img0: d_dets is the lane's)
      a.counts2 = args->counts_after_dets
                      ? reinterpret_cast<int*>(d_dets + (size_t)(c->call_B - c->lane_img0) * args->max_det * (6 + c->nm)) +
                            c->lane_img0
                      : nullptr;
      a.A = c->A; a.kstride = c->kstride; a.nm = c->nm; a.max_det = args->max_det; a.max_nms = args->max_nms;
      a.agnostic = args->agnostic; a.B = B; a.nc = c->nc;
      a.max_wh = args->max_wh; a.img_h = (float)c->cH; a.img_w = (float)c->cW;
      a.iou = args->iou;
      // low conf (the validator's 0.001): thousands of candidates per image; sort their keys over several
      // workgroups per image first (conf is part of the graph key: the predict default 0.25 never launches these)
      if (args->conf < kPresortConf && c->kstride >= 16384) {
        a.keys2 = c->scratch<unsigned long long>(c->off_keys2, (size_t)c->kstride * 8);
        a.presorted = 1;
        e = ym_launch_nms_presort(a, st);
        if (e != hipSuccess) break;
      }
      e = ym_launch_nms(a, st);
      break;
    }
    default:
      return fail(YM_EBLOB, "unknown op kind %d", r[0]);
  }
  if (e != hipSuccess) return fail(YM_EHIP, "launch of op %s failed: %s", op.name, hipGetErrorString(e));
  return YM_OK;
}

int check_call(ym_ctx* c, const float* d_in, int B, int H, int W, const ym_infer_args* args, float* d_dets,
               int* d_counts) {
  if (!c) return fail(YM_EINVAL, "null context");
  if (!c->loaded) return fail(YM_ESTATE, "ym_infer before ym_load_weights");
  if (!d_in || !d_dets || !d_counts || !args) return fail(YM_EINVAL, "null pointer argument");
  if (B < 1 || H < 32 || W < 32 || H % 32 || W % 32)
    return fail(YM_EINVAL, "input shape (%d,3,%d,%d): H and W must be positive multiples of 32", B, H, W);
  if (args->max_det < 1 || args->max_nms < 1) return fail(YM_EINVAL, "max_det/max_nms must be >= 1");
  if (args->max_det > 1024) return fail(YM_EINVAL, "max_det %d > 1024 is not supported", args->max_det);
  if (args->counts_after_dets != 0 && args->counts_after_dets != 1) return fail(YM_EINVAL, "counts_after_dets is 0 or 1");
  c->call_B = B;  // (launch_forward sets it again; eager per-op paths launch the NMS op directly)
  return YM_OK;
}

}  // namespace

extern "C" {

int ym_version(void) { return 1; }
int ym_num_conv_cfgs(int dtype) {  // public dtype codes (ym_model_desc): 1 f16, 2 f32, 3 i8, 4 f8, 5 x3
  if (dtype < 1 || dtype > 5) return YM_EINVAL;
  static const int dt[6] = {0, YM_DT_F16, YM_DT_F32, YM_DT_I8, YM_DT_F8, YM_DT_X3};
  return ym_conv_num_cfgs_dt(dt[dtype]);
}

const char* ym_last_error(void) { return g_err.c_str(); }
int ym_set_debug(int key, int value) {
  if (key < YM_DBG_NMS || key > YM_DBG_CONV_CFG) return fail(YM_EINVAL, "unknown debug key %d", key);
  return ym_debug_set(key, value);
}

int ym_create(int device, const ym_model_desc* desc, ym_ctx** out) {
  if (!out) return fail(YM_EINVAL, "null out");
  int n = 0;
  HIPCK(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(YM_EINVAL, "device %d out of range (%d devices)", device, n);
  HIPCK(hipSetDevice(device));
  ym_ctx* c = new ym_ctx();
  c->device = device;
  if (desc) c->desc = *desc;
  hipError_t e = hipStreamCreateWithFlags(&c->cap_stream, hipStreamNonBlocking);
  for (int l = 1; l < kMaxLanes && e == hipSuccess; ++l) e = hipStreamCreateWithFlags(&c->lane_streams[l], hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming);
  // ym_input_max's ctl region (slots, ticket, partials: YM_CTL_BYTES) at 0, broadcast control words at 8 KB
  if (e == hipSuccess) e = hipMalloc(&c->d_misc, kMiscBytes);
  if (e == hipSuccess) e = hipMemset(c->d_misc, 0, kMiscBytes);
  for (int l = 1; l < kMaxLanes && e == hipSuccess; ++l) e = hipEventCreateWithFlags(&c->join_ev[l], hipEventDisableTiming);
  if (e != hipSuccess) {
    delete c;
    return fail(YM_EHIP, "hipStreamCreate/hipEventCreate: %s", hipGetErrorString(e));
  }
  *out = c;
  return YM_OK;
}


// Static branch schedule (one-lane forwards): op i depends on every earlier op that writes a buffer it reads
// (buffer granularity; the planner never rewrites a buffer region within a forward, so RAW is the only hazard).
// Ops go in program order onto up to kMaxLanes streams: an op continues the stream of its latest dependency when
// that dependency is the stream's tail, else opens an unused stream, else joins the stream whose tail is oldest.
// Cross-stream dependencies become event waits (skipped when already implied by an earlier wait).  The Detect-head
// chains of P3/P4 then run beside the neck's latency-bound 40x40/20x20 layers.
static void build_schedule(ym_ctx* c) {
  const int nop = (int)c->ops.size(), nbuf = (int)c->bufs.size();
  const int P_DEC = nbuf, P_OUT = nbuf + 1;  // pseudo buffers: decode scratch, detections
  auto rw = [&](const Op& o, std::vector<int>& rd, std::vector<int>& wr) {
    const int32_t* r = o.r;
    rd.clear(); wr.clear();
    switch (r[0]) {
      case OP_INPUT: wr.push_back(c->input_buf); break;
      case OP_CONV: rd.push_back(r[6]); if (r[10] >= 0) rd.push_back(r[10]); if (r[17] >= 0) rd.push_back(r[17]);
                    wr.push_back(r[13]); break;
      case OP_DW: case OP_ATTN: case OP_REQ: rd.push_back(r[6]); wr.push_back(r[13]); break;
      case OP_SPPF: rd.push_back(r[13]); wr.push_back(r[13]); break;
      case OP_DECODE: rd.push_back(c->anchor_buf); wr.push_back(P_DEC); break;
      case OP_NMS: rd.push_back(P_DEC); rd.push_back(c->anchor_buf); wr.push_back(P_OUT); break;
      default: rd.push_back(-2); break;  // unknown: serialise behind everything
    }
  };
  const int S = kMaxLanes;
  c->br_of.assign(nop, 0);
  c->br_wait.assign(nop, {});
  c->br_rec.assign(nop, 0);
  std::vector<std::vector<int>> writers(nbuf + 2);
  std::vector<int> tail(S, -1);
  std::vector<std::vector<int>> known(S, std::vector<int>(S, -1));  // known[s][t]: ops of stream t done before s
  std::vector<std::vector<int>> snap(nop);                          // known vector of an op's stream after it
  std::vector<int> rd, wr;
  int used = 1;
  // YM_BRANCHES=1..4; default 4 streams for f16 detect plans, serial otherwise.  tools/branch_ab.sh on MI355X (one
  // box, bench.py device img/s, serial -> 4 streams): yolo11s f16 B=8 8.06k -> 8.51k, yolo11n f16 12.1k -> 13.0k (the
  // Detect-head chains of one level overlap the neck's 20x20 / 40x40 layers, whose launches leave most CUs idle), but
  // yolo11s-seg f16 B=4 4.35k -> 3.84k, yolo11n int8 8.62k -> 7.39k and fp8 9.25k -> 7.87k (their head / requant /
  // float-island kernels contend with the neck instead of filling idle CUs).  Round 3, x3 detect plans: yolo11s B=8
  // 4.47k -> 4.68k predict img/s, yolo11n device 6.88k -> 7.31k: on by default too.
  const char* env = getenv("YM_BRANCHES");
  const int def = (c->dtype == YM_DT_F16 || c->dtype == YM_DT_X3) && c->task == 0 ? S : 1;
  const int maxs = env && *env ? (atoi(env) < 1 ? 1 : (atoi(env) > S ? S : atoi(env))) : def;
  // YM_SCHED=crit: continue the stream of the dependency expected to finish LAST (a per-op time estimate at
  // 640², B = 8: ~6 us per launch plus MACs at ~40 TMAC/s), instead of the latest dependency in program order — a
  // join then waits on the other streams' earlier producers, and the slowest chain flows straight into its consumer
  // without a cross-queue wait (the kernel trace shows ~10 us idle at such joins, e.g. before decode)
  const char* sched = getenv("YM_SCHED");
  const bool crit = sched && !strcmp(sched, "crit");
  std::vector<double> fin(nop, 0.0), sfin(S, 0.0);
  auto est_us = [&](const Op& o) {
    const int32_t* r = o.r;
    double macs = 0;
    if (r[0] == OP_CONV && r[13] >= 0 && r[13] < nbuf) {
      const int f = c->bufs[r[13]].f > 0 ? c->bufs[r[13]].f : 8;  // output stride (head rows: level stride unknown)
      const double px = 8.0 * (640.0 / f) * (640.0 / f);
      macs = px * r[1] * r[1] * (double)r[3] * r[4] * (r[30] ? 2 : 1);
    }
    return 6.0 + macs / 40e6;
  };
  for (int i = 0; i < nop; ++i) {
    rw(c->ops[i], rd, wr);
    std::vector<int> deps;
    bool all = false;
    for (int b : rd) {
      if (b == -2) all = true;
      else if (b >= 0 && b < nbuf + 2) deps.insert(deps.end(), writers[b].begin(), writers[b].end());
    }
    if (all) for (int j = 0; j < i; ++j) deps.push_back(j);
    int jmax = -1;
    for (int j : deps) jmax = j > jmax ? j : jmax;
    int s = -1;
    if (crit) {  // the stream tail among the dependencies with the latest estimated finish
      double best = -1;
      for (int j : deps)
        if (tail[c->br_of[j]] == j && fin[j] > best) { best = fin[j]; s = c->br_of[j]; }
    }
    if (s < 0 && jmax >= 0 && tail[c->br_of[jmax]] == jmax) s = c->br_of[jmax];
    if (s < 0 && jmax >= 0 && used < maxs) s = used++;
    if (s < 0) {  // the stream whose tail is oldest
      s = 0;
      for (int t = 1; t < used; ++t) if (tail[t] < tail[s]) s = t;
    }
    if (i == 0) s = 0;
    for (int j : deps) {
      const int t = c->br_of[j];
      if (t == s || known[s][t] >= j) continue;
      c->br_wait[i].push_back(j);
      c->br_rec[j] = 1;
      known[s][t] = j;
      for (int u = 0; u < S; ++u) if (snap[j][u] > known[s][u]) known[s][u] = snap[j][u];
    }
    double start = sfin[s];
    for (int j : deps) start = fin[j] > start ? fin[j] : start;
    fin[i] = sfin[s] = start + est_us(c->ops[i]);
    c->br_of[i] = s;
    tail[s] = i;
    known[s][s] = i;
    snap[i] = known[s];
    for (int b : wr) if (b >= 0 && b < nbuf + 2) writers[b].push_back(i);
  }
  c->nbr = used;
}

// OCP e4m3 (gfx950 fp8) code -> value: the fp8 plan's stem weights, re-laid out as fp32 (exact)
static float e4m3_value(uint8_t b) {
  const int e = (b >> 3) & 15, m = b & 7;
  const float v = e == 0 ? ldexpf((float)m, -9) : ((e == 15 && m == 7) ? NAN : ldexpf((float)(8 + m), e - 10));
  return (b & 0x80) ? -v : v;
}

// Structural check of a parsed plan before it is committed to a context: buffer ids and channel views
// [coff, coff + C) of every op record inside their buffers, every weight / bias / quantisation record inside the
// weight section.  The kernels index device memory with these values, so a malformed blob must fail here
// (YM_EBLOB), never inside a launch.
static int validate_plan(const std::vector<BufDesc>& bufs, const std::vector<Op>& ops, int dtype, size_t wbytes,
                         int input_buf) {
  const int nbuf = (int)bufs.size();
  for (int i = 0; i < nbuf; ++i)
    if (bufs[i].C <= 0 || bufs[i].C > (1 << 16) || bufs[i].f < 0 || bufs[i].f > 64)
      return fail(YM_EBLOB, "buffer %d: bad geometry (C %d, f %d)", i, bufs[i].C, bufs[i].f);
  // (x3 plans: Kpad counts the fp16 [hi | lo] storage K of the pair-chunk weight rows; their fp32 stem rows are
  // checked again where they are read)
  const size_t esz = dtype == YM_DT_F32 ? 4 : ((dtype == YM_DT_F16 || dtype == YM_DT_X3) ? 2 : 1);
  for (const Op& o : ops) {
    const int32_t* r = o.r;
    auto buf_ok = [&](int b, bool opt) { return (opt && b == -1) || (b >= 0 && b < nbuf); };
    auto w_ok = [&](int32_t off, size_t n) { return (size_t)(uint32_t)off + n <= wbytes; };
    // a channel view [coff, coff + C) of buffer b (b == -1: absent, when optional)
    auto view_ok = [&](int b, int coff, int C, bool opt) {
      if (opt && b == -1) return true;
      return buf_ok(b, false) && coff >= 0 && C > 0 && (long)coff + C <= bufs[b].C;
    };
    bool ok = true;
    const size_t qrec = sizeof(QRec);
    switch (r[0]) {
      case OP_INPUT: case OP_DECODE: case OP_NMS: break;  // no operands besides the header's input/anchor buffers
      case OP_CONV: {
        const int N = r[4], Kpad = r[21], fused = r[30];
        const int Nout = fused ? r[27] : N;  // the channels the launch writes (a fused pair: its second conv's)
        const int Cd = r[16] ? Nout / 4 : Nout;  // pixel shuffle (ConvTranspose2d 2x2): N/4 channels per pixel
        const int C1 = r[10] >= 0 ? r[12] : 0;
        ok = N > 0 && Kpad > 0 && Kpad <= (1 << 16) && r[3] == r[8] + C1 && view_ok(r[6], r[7], r[8], false) &&
             view_ok(r[10], r[11], r[12], true) && view_ok(r[13], r[14], Cd, false) &&
             view_ok(r[17], r[18], Nout, true) && (r[6] != input_buf || (r[7] == 0 && r[10] == -1)) &&
             w_ok(r[19], (size_t)N * Kpad * esz) && w_ok(r[20], (size_t)N * 4);
        if (ok && ym_dt_q8(dtype)) ok = w_ok(r[22], qrec) && w_ok(r[23], (size_t)N * 4) && w_ok(r[24], (size_t)N * 4);
        else if (ok && r[24] > 0) ok = w_ok(r[24] - 1, (size_t)10 * r[3] * 4);  // fused depthwise weights + bias
        if (ok && fused) {
          const int N2 = r[27], K2 = r[29];
          ok = N2 > 0 && K2 > 0 && K2 <= (1 << 16) && buf_ok(r[31], false) && w_ok(r[25], (size_t)N2 * K2 * 2) &&
               w_ok(r[26], (size_t)N2 * 4);
        }
        break;
      }
      case OP_DW: case OP_ATTN: {
        const int C = r[3];
        // attention: the (q, k, v) channels of every head after q_coff; the output slice is C wide
        const int Cin = r[0] == OP_ATTN ? r[4] * (2 * r[5] + r[9]) : C;
        ok = C > 0 && view_ok(r[6], r[7], Cin, false) && view_ok(r[13], r[14], C, false) &&
             (r[0] == OP_DW || (r[4] > 0 && r[4] * r[9] == C)) &&
             w_ok(r[19], (size_t)9 * C * (ym_dt_q8(dtype) ? 1 : 4)) && w_ok(r[20], (size_t)C * 4);
        if (ok && ym_dt_q8(dtype)) ok = w_ok(r[22], qrec) && w_ok(r[23], (size_t)C * 4);
        break;
      }
      case OP_SPPF: ok = r[3] > 0 && view_ok(r[13], r[7], 4 * r[3], false); break;  // y0 and the 3 pooled slices
      case OP_REQ:
        ok = r[3] > 0 && view_ok(r[6], r[7], r[3], false) && view_ok(r[13], r[14], r[3], false) && w_ok(r[22], qrec);
        break;
      default: return fail(YM_EBLOB, "op %s: unknown op kind %d", o.name, r[0]);
    }
    if (!ok) return fail(YM_EBLOB, "op %s: buffer id, channel view or weight range out of bounds", o.name);
  }
  return YM_OK;
}

int ym_load_weights(ym_ctx* c, const void* blob, size_t bytes) {
  if (!c || !blob) return fail(YM_EINVAL, "null argument");
  HIPCK(hipSetDevice(c->device));
  const int32_t* h = static_cast<const int32_t*>(blob);
  if (bytes < kHdr * 4 || h[0] != kMagic || h[1] != 1) return fail(YM_EBLOB, "bad blob magic/version");
  // everything is parsed into locals and validated; the context changes only once the whole blob checks out
  const int nbuf = h[11], nop = h[12];
  if (nbuf < 1 || nbuf > 4096 || nop < 1 || nop > 4096) return fail(YM_EBLOB, "bad buffer/op counts (%d, %d)", nbuf, nop);
  const size_t wbytes = (size_t)(uint32_t)h[13] | ((size_t)(uint32_t)h[14] << 32);
  const size_t need = (size_t)kHdr * 4 + (size_t)nbuf * kBufRec * 4 + (size_t)nop * (kOpRec * 4 + kNameLen);
  const size_t woff = align_up(need, 256);
  if (wbytes > bytes || bytes < woff + wbytes) return fail(YM_EBLOB, "blob truncated (%zu < %zu)", bytes, woff + wbytes);
  const int dtype = h[2];
  if (dtype != YM_DT_F16 && !ym_dt_f32s(dtype) && !ym_dt_q8(dtype)) return fail(YM_EBLOB, "unknown dtype %d", dtype);
  const int task = h[3], nc = h[4], nm = h[5], reg_max = h[6], nl = h[7];
  if (nl < 1 || nl > 4) return fail(YM_EBLOB, "bad level count");
  if (nc < 1 || nc > 128 || nm < 0 || nm > 64 || reg_max < 1 || reg_max > 64)
    return fail(YM_EBLOB, "bad head geometry (nc %d, nm %d, reg_max %d)", nc, nm, reg_max);
  for (int l = 0; l < nl; ++l)
    if (h[8 + l] < 1 || h[8 + l] > 64) return fail(YM_EBLOB, "bad stride %d", h[8 + l]);
  const ym_model_desc& want = c->desc;  // what the creator expects (0 = any)
  if (want.task && want.task != task + 1)
    return fail(YM_EBLOB, "blob task %s, context created for %s", task ? "segment" : "detect",
                want.task == YM_TASK_SEGMENT ? "segment" : "detect");
  if (want.dtype && want.dtype != dtype + 1) return fail(YM_EBLOB, "blob dtype %d, context created for %d", dtype + 1, want.dtype);
  if (want.scale && h[19] && want.scale != h[19])
    return fail(YM_EBLOB, "blob scale '%c', context created for '%c'", (char)h[19], (char)want.scale);
  const int input_buf = h[15], anchor_buf = h[16], proto_buf = h[17];
  if (input_buf < 0 || input_buf >= nbuf || anchor_buf < 0 || anchor_buf >= nbuf)
    return fail(YM_EBLOB, "bad input/anchor buffer ids");
  if (task == 1 && (proto_buf < 0 || proto_buf >= nbuf)) return fail(YM_EBLOB, "segment plan without proto buffer");
  const int32_t* bp = h + kHdr;
  std::vector<BufDesc> bufs(nbuf);
  for (int i = 0; i < nbuf; ++i) bufs[i] = BufDesc{bp[i * kBufRec], bp[i * kBufRec + 1], bp[i * kBufRec + 2]};
  const int32_t* op = bp + (size_t)nbuf * kBufRec;
  const char* names = reinterpret_cast<const char*>(op + (size_t)nop * kOpRec);
  std::vector<Op> ops(nop);
  for (int i = 0; i < nop; ++i) {
    memcpy(ops[i].r, op + (size_t)i * kOpRec, kOpRec * 4);
    memcpy(ops[i].name, names + (size_t)i * kNameLen, kNameLen);
    ops[i].name[kNameLen - 1] = 0;
  }
  int rc = validate_plan(bufs, ops, dtype, wbytes, input_buf);
  if (rc) return rc;
  // commit: a reload drops the previous plan's workspace, graphs and per-shape tile tables (they index its ops and
  // buffers); the weights are replaced below
  c->loaded = false;
  c->clear_graphs();
  if (c->d_arena || c->d_weights) HIPCK(hipDeviceSynchronize());  // no launch may still use the old plan's memory
  if (c->d_arena) HIPCK(hipFree(c->d_arena));
  c->d_arena = nullptr;
  c->arena_bytes = 0;
  c->cB = c->cH = c->cW = 0;
  c->buf_off.clear();
  c->cfgs.clear();
  c->dtype = dtype;
  c->task = task; c->nc = nc; c->nm = nm; c->reg_max = reg_max; c->nl = nl;
  for (int l = 0; l < nl; ++l) c->strides[l] = h[8 + l];
  c->input_buf = input_buf; c->anchor_buf = anchor_buf; c->proto_buf = proto_buf; c->no = h[18];
  c->bufs = std::move(bufs);
  c->ops = std::move(ops);
  c->blob_host.assign(static_cast<const char*>(blob), static_cast<const char*>(blob) + bytes);  // ym_broadcast_weights
  build_schedule(c);
  while (c->op_ev.size() < c->ops.size()) {
    hipEvent_t ev;
    HIPCK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    c->op_ev.push_back(ev);
  }
  c->clear_graphs();
  if (c->d_weights) HIPCK(hipFree(c->d_weights));
  c->d_weights = nullptr;
  // The stem conv's weights, re-laid out on the host as fp32 [27][N] (tap-major: (ky, kx, c), N contiguous) so the
  // stem kernel reads them with wave-uniform (scalar) loads; the blob packs them as [N][Kpad] GEMM rows with the
  // 3 input channels padded to 8 per tap.  int8 plans keep the integer weight values, fp8 plans the e4m3 values
  // (both exact in fp32).
  std::vector<float> wstem;
  for (const Op& o : c->ops) {
    if (o.r[0] != OP_CONV || o.r[6] != c->input_buf) continue;
    const int N = o.r[4], Kpad = o.r[21];
    if (o.r[1] != 3 || o.r[3] != 8 || Kpad < 72) return fail(YM_EBLOB, "op %s: unexpected stem geometry", o.name);
    const char* w = static_cast<const char*>(blob) + woff + (size_t)(uint32_t)o.r[19];
    const size_t esz = ym_dt_f32s(c->dtype) ? 4 : (c->dtype == YM_DT_F16 ? 2 : 1);
    if ((size_t)(uint32_t)o.r[19] + (size_t)N * Kpad * esz > wbytes) return fail(YM_EBLOB, "stem weights out of range");
    wstem.assign((size_t)27 * N, 0.f);
    for (int n = 0; n < N; ++n)
      for (int t = 0; t < 27; ++t) {
        const size_t i = (size_t)n * Kpad + (t / 3) * 8 + t % 3;
        float v;
        if (ym_dt_f32s(c->dtype)) memcpy(&v, w + 4 * i, 4);
        else if (c->dtype == YM_DT_F16) { _Float16 h16; memcpy(&h16, w + 2 * i, 2); v = (float)h16; }
        else if (c->dtype == YM_DT_F8) v = e4m3_value(reinterpret_cast<const uint8_t*>(w)[i]);
        else v = (float)reinterpret_cast<const int8_t*>(w)[i];
        wstem[(size_t)t * N + n] = v;
      }
    break;
  }
  // int8 plans: per 3x3 conv the [9][N] int32 tap sums of its weights (ConvArgs::wtap: the LDS-DMA kernels' padding
  // correction), behind the stem weights
  std::vector<int32_t> wtap;
  c->off_wtap.assign(c->ops.size(), 0);
  if (dtype == YM_DT_I8) {
    for (size_t i = 0; i < c->ops.size(); ++i) {
      const Op& o = c->ops[i];
      if (o.r[0] != OP_CONV || o.r[6] == c->input_buf || o.r[1] != 3) continue;
      const int N = o.r[4], Kpad = o.r[21], cin = o.r[3], cs = (cin + 15) / 16 * 16;
      if (9 * cs > Kpad || (size_t)(uint32_t)o.r[19] + (size_t)N * Kpad > wbytes) continue;
      const int8_t* w = reinterpret_cast<const int8_t*>(static_cast<const char*>(blob) + woff + (size_t)(uint32_t)o.r[19]);
      c->off_wtap[i] = wtap.size() * 4 + 1;  // + 1: 0 means none (relative to off_wtap0, 4-byte units * 4)
      for (int t = 0; t < 9; ++t)
        for (int n = 0; n < N; ++n) {
          int32_t sum = 0;
          for (int k = 0; k < cs; ++k) sum += w[(size_t)n * Kpad + t * cs + k];
          wtap.push_back(sum);
        }
    }
  }
  c->off_wstem = align_up(wbytes, 256);
  c->off_wtap0 = align_up(c->off_wstem + wstem.size() * sizeof(float), 256);
  const size_t dbytes = c->off_wtap0 + wtap.size() * sizeof(int32_t);
  hipError_t e = hipMalloc(&c->d_weights, dbytes ? dbytes : 256);
  if (e != hipSuccess) return fail(YM_ENOMEM, "weights hipMalloc(%zu): %s", dbytes, hipGetErrorString(e));
  HIPCK(hipMemcpy(c->d_weights, static_cast<const char*>(blob) + woff, wbytes, hipMemcpyHostToDevice));
  if (!wstem.empty())
    HIPCK(hipMemcpy(c->d_weights + c->off_wstem, wstem.data(), wstem.size() * sizeof(float), hipMemcpyHostToDevice));
  if (!wtap.empty())
    HIPCK(hipMemcpy(c->d_weights + c->off_wtap0, wtap.data(), wtap.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  c->wbytes = wbytes;
  c->loaded = true;
  return YM_OK;
}

// Lane split of a B-image batch: L = clamp(args->lanes, 1, kMaxLanes) slices of ceil(B / L) images (0 = 1 lane).
static void lane_split(const ym_infer_args* args, int B, int& L, int& Bl) {
  L = args->lanes < 1 ? 1 : (args->lanes > kMaxLanes ? kMaxLanes : args->lanes);
  if (L > B) L = B;
  Bl = (B + L - 1) / L;
  L = (B + Bl - 1) / Bl;
}

// YM_DBG_CHAIN = 1 (ym_set_debug, or YM_CHAIN=1 in the environment; verdict r5 item 1): op i and op i+1 as ONE persistent launch (csrc/ym_conv_dma.hip
// conv_dma_chain) where both are x3 3x3 convs on the same LDS-DMA configuration, op i+1 reads op i's output and waits
// for nothing else, and both run on the main stream (one chain kernel in flight at a time).  Returns 1 when launched.
static int try_chain(ym_ctx* c, size_t i, int B, const float* d_in, const ym_infer_args* args, hipStream_t st,
                     int& rc) {
  rc = YM_OK;
  if (ym_debug_get(YM_DBG_CHAIN) != 1 || c->dtype != YM_DT_X3 || i + 1 >= c->ops.size() || c->lane != 0) return 0;
  const Op &o0 = c->ops[i], &o1 = c->ops[i + 1];
  if (o0.r[0] != OP_CONV || o1.r[0] != OP_CONV || o0.r[30] || o1.r[30]) return 0;
  if (c->nbr > 1 && (c->br_of[i] != 0 || c->br_of[i + 1] != 0 || !c->br_wait[i + 1].empty())) return 0;
  const int cf0 = c->op_cfg((long)i, B), cf1 = c->op_cfg((long)i + 1, B);
  const int dma = cf0 - 17;  // LDS-DMA ids follow the 17 first-generation configurations (csrc/ym_conv.hip)
  if (cf0 != cf1 || (dma != 8 && dma != 13 && dma != 26)) return 0;
  ConvArgs a0{}, a1{};
  int f0 = 0, f1 = 0;
  if ((rc = conv_args(c, o0, B, d_in, args->in_eps, a0, f0)) || (rc = conv_args(c, o1, B, d_in, args->in_eps, a1, f1)))
    return 1;
  if (f0 || f1 || a0.nchw) return 0;
  const hipError_t e = ym_launch_conv_dma_chain(a0, a1, dma, reinterpret_cast<int*>(c->d_arena + c->off_chain),
                                                kChainCtl, st);
  if (e == hipErrorInvalidValue) return 0;  // shapes the chain kernel does not take: two launches
  if (e != hipSuccess) rc = fail(YM_EHIP, "chain launch of %s + %s: %s", o0.name, o1.name, hipGetErrorString(e));
  else ym_debug_add(YM_DBG_CHAIN_LAUNCHES, 1);
  return 1;
}

// YM_DBG_STEMFUSE = 1 (verdict r5 item 5): the x3 stem (op i) and the fused 3x3 s2 -> 1x1 pair that
// reads its output (op i + 1: model.1 -> model.2.cv1) as ONE launch (csrc/ym_stem_fused.hip): the stem's output is
// never stored.  Only where nothing else reads that output and op i + 1 waits for nothing else.  Returns 1 when
// launched.
static int try_stem_fuse(ym_ctx* c, size_t i, int B, const float* d_in, const ym_infer_args* args, hipStream_t st,
                         int& rc) {
  rc = YM_OK;
  if (ym_debug_get(YM_DBG_STEMFUSE) != 1 || c->dtype != YM_DT_X3 || i + 1 >= c->ops.size()) return 0;
  const Op &o0 = c->ops[i], &o1 = c->ops[i + 1];
  if (o0.r[0] != OP_CONV || o1.r[0] != OP_CONV || o0.r[6] != c->input_buf || !o1.r[30] || o1.r[6] != o0.r[13])
    return 0;
  if (c->nbr > 1 && (c->br_of[i] != c->br_of[i + 1] || !c->br_wait[i + 1].empty())) return 0;
  const int sb = o0.r[13];
  for (size_t j = 0; j < c->ops.size(); ++j) {  // the stem's output: op i + 1 must be its only reader
    if (j == i + 1) continue;
    const int32_t* r = c->ops[j].r;
    bool reads = false;
    switch (r[0]) {
      case OP_CONV: reads = r[6] == sb || r[10] == sb || r[17] == sb; break;
      case OP_DW: case OP_ATTN: case OP_REQ: reads = r[6] == sb; break;
      case OP_SPPF: reads = r[13] == sb; break;
      default: break;
    }
    if (reads) return 0;
  }
  ConvArgs a0{}, a1{};
  int f0 = 0, f1 = 0;
  if ((rc = conv_args(c, o0, B, d_in, args->in_eps, a0, f0)) || (rc = conv_args(c, o1, B, d_in, args->in_eps, a1, f1)))
    return 1;
  if (f0 || f1) return 0;
  const hipError_t e = ym_launch_stem_down_x3(a0, a1, st);
  if (e == hipErrorInvalidValue) return 0;
  if (e != hipSuccess) rc = fail(YM_EHIP, "fused stem launch of %s + %s: %s", o0.name, o1.name, hipGetErrorString(e));
  return 1;
}

// Launch one forward: the input statistics over the WHOLE batch (LoadTensor's /255 rule is a batch-wide max), then
// every other op per lane on its image slice.  With fork/join events the lanes are parallel graph branches when
// `st` is capturing; eagerly (no capture) they run on the lane streams concurrently as well.
static int launch_forward(ym_ctx* c, const float* d_in, int B, const ym_infer_args* args, float* d_dets,
                          int* d_counts, hipStream_t st) {
  int L, Bl, rc;
  lane_split(args, B, L, Bl);
  c->call_B = B;
  c->lane = 0;
  c->lane_img0 = 0;
  if (L == 1 && c->nbr > 1) {  // one lane: the branch schedule (build_schedule)
    hipStream_t bs[kMaxLanes] = {st};
    for (int s = 1; s < kMaxLanes; ++s) bs[s] = c->lane_streams[s];
    for (size_t i = 0; i < c->ops.size(); ++i) {
      const int s = c->br_of[i];
      for (int j : c->br_wait[i]) HIPCK(hipStreamWaitEvent(bs[s], c->op_ev[j], 0));
      c->lane = s;  // split-K slab / counter region of this stream
      if (try_stem_fuse(c, i, B, d_in, args, bs[s], rc) || try_chain(c, i, B, d_in, args, bs[s], rc)) {  // ops i, i + 1
        c->lane = 0;
        if (rc) return rc;
        if (c->br_rec[i]) HIPCK(hipEventRecord(c->op_ev[i], bs[s]));
        ++i;
      } else {
        rc = launch_op(c, c->ops[i], B, d_in, args, d_dets, d_counts, bs[s]);
        c->lane = 0;
      }
      if (rc) return rc;
      if (c->br_rec[i]) HIPCK(hipEventRecord(c->op_ev[i], bs[s]));
    }
    for (int s = 1; s < c->nbr; ++s) {  // every branch joins back into the caller's stream
      HIPCK(hipEventRecord(c->join_ev[s], bs[s]));
      HIPCK(hipStreamWaitEvent(st, c->join_ev[s], 0));
    }
    return YM_OK;
  }
  size_t o = 0;
  for (o = 0; o < c->ops.size() && c->ops[o].r[0] == OP_INPUT; ++o)
    if ((rc = launch_op(c, c->ops[o], B, d_in, args, d_dets, d_counts, st))) return rc;
  if (L > 1) HIPCK(hipEventRecord(c->fork_ev, st));
  const size_t in_img = (size_t)3 * c->cH * c->cW, det_img = (size_t)args->max_det * (6 + c->nm);
  for (int l = 0; l < L; ++l) {
    hipStream_t ls = l == 0 ? st : c->lane_streams[l];
    if (l > 0) HIPCK(hipStreamWaitEvent(ls, c->fork_ev, 0));
    c->lane = l;
    c->lane_img0 = l * Bl;
    const int nb = B - l * Bl < Bl ? B - l * Bl : Bl;
    for (size_t i = o; i < c->ops.size(); ++i) {
      if (L == 1 && (try_stem_fuse(c, i, nb, d_in, args, ls, rc) || try_chain(c, i, nb, d_in, args, ls, rc))) {
        ++i;
        if (!rc) continue;
      } else {
        rc = launch_op(c, c->ops[i], nb, d_in + c->lane_img0 * in_img, args, d_dets + c->lane_img0 * det_img,
                       d_counts + c->lane_img0, ls);
      }
      if (rc) {
        c->lane = c->lane_img0 = 0;
        return rc;
      }
    }
    if (l > 0) {
      HIPCK(hipEventRecord(c->join_ev[l], ls));
      HIPCK(hipStreamWaitEvent(st, c->join_ev[l], 0));
    }
  }
  c->lane = c->lane_img0 = 0;
  return YM_OK;
}

int ym_infer(ym_ctx* c, const float* d_in, int B, int H, int W, const ym_infer_args* args, float* d_dets,
             int* d_counts, void* stream) {
  int rc = check_call(c, d_in, B, H, W, args, d_dets, d_counts);
  if (rc) return rc;
  HIPCK(hipSetDevice(c->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  rc = ensure_workspace(c, B, H, W);
  if (rc) return rc;
  if ((rc = c->order_after_last(st))) return rc;
  if (!args->use_graph) {
    if (!c->fwd_ev) HIPCK(hipEventCreateWithFlags(&c->fwd_ev, hipEventDisableTiming));
    if ((rc = launch_forward(c, d_in, B, args, d_dets, d_counts, st))) return rc;
    HIPCK(hipEventRecord(c->fwd_ev, st));
    c->last_ev = c->fwd_ev;
    c->last_st = st;
    return YM_OK;
  }
  GraphKey key;
  memset(&key, 0, sizeof(key));
  key.B = B; key.H = H; key.W = W; key.in = d_in; key.dets = nullptr; key.counts = d_counts; key.args = *args;
  GraphKey key_d = key;  // the key of a graph whose NMS nodes could not be re-pointed
  key_d.dets = d_dets;
  for (auto& g : c->graphs) {
    if (g.key == key || g.key == key_d) {
      // re-pointable: new rows through the NMS nodes' parameters.  A launch already queued keeps the parameters it
      // was launched with (hipGraphExecKernelNodeSetParams changes later launches only:
      // tests/test_gpu_kernels.py test_repointed_graph_rows_with_no_sync_between_calls), so no wait here — an
      // asynchronous predict() loop enqueues the next forward while the previous one runs
      if (g.key == key && g.dets != d_dets && (rc = repoint_dets(g, d_dets))) return rc;
      HIPCK(hipGraphLaunch(g.exec, st));
      HIPCK(hipEventRecord(g.done, st));
      c->last_ev = g.done;
      c->last_st = st;
      return YM_OK;
    }
  }
  if (c->graphs.size() >= kMaxGraphs) {  // evict the oldest capture once its last replay has drained
    c->retire(c->graphs.front());
    c->graphs.erase(c->graphs.begin());
  }
  // capture on the private stream (lane streams join through the fork event), replay on the caller's stream
  HIPCK(hipStreamBeginCapture(c->cap_stream, hipStreamCaptureModeRelaxed));
  if ((rc = launch_forward(c, d_in, B, args, d_dets, d_counts, c->cap_stream))) {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(c->cap_stream, &g);
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  GraphEntry ge;
  HIPCK(hipStreamEndCapture(c->cap_stream, &ge.graph));
  hipError_t e = hipGraphInstantiate(&ge.exec, ge.graph, nullptr, nullptr, 0);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ge.done, hipEventDisableTiming);
  if (e != hipSuccess) {
    retire_graph(ge);
    return fail(YM_EHIP, "graph instantiate: %s", hipGetErrorString(e));
  }
  ge.dets = d_dets;
  static const bool no_repoint = [] { const char* v = getenv("YM_GRAPH_REPOINT"); return v && *v == '0'; }();
  ge.key = (!no_repoint && find_nms_nodes(ge)) ? key : key_d;
  c->graphs.push_back(ge);
  HIPCK(hipGraphLaunch(ge.exec, st));
  HIPCK(hipEventRecord(ge.done, st));
  c->last_ev = ge.done;
  c->last_st = st;
  return YM_OK;
}

int ym_input_max(ym_ctx* c, const float* d_in, size_t n, float* d_max, void* stream) {
  if (!c || !d_in || !d_max || n == 0) return fail(YM_EINVAL, "bad ym_input_max arguments");
  HIPCK(hipSetDevice(c->device));
  const hipError_t e = ym_launch_input_max(d_in, (long)n, reinterpret_cast<float*>(c->d_misc), d_max,
                                           static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return fail(YM_EHIP, "input max: %s", hipGetErrorString(e));
  return YM_OK;
}

int ym_calibrate(ym_ctx* c, const float* d_in, int B, int H, int W, const ym_infer_args* args, float* d_dets,
                 int* d_counts, float* const* d_raw, int n_ops, void* stream) {
  int rc = check_call(c, d_in, B, H, W, args, d_dets, d_counts);
  if (rc) return rc;
  if (c->dtype != YM_DT_F32) return fail(YM_ESTATE, "ym_calibrate needs an f32 (parity) plan");
  if (!d_raw || n_ops != (int)c->ops.size()) return fail(YM_EINVAL, "d_raw must hold %zu entries", c->ops.size());
  HIPCK(hipSetDevice(c->device));
  if ((rc = ensure_workspace(c, B, H, W))) return rc;
  if ((rc = c->order_after_last(static_cast<hipStream_t>(stream)))) return rc;
  ym_infer_args one = *args;
  one.lanes = 1;
  c->calib_raw = d_raw;
  rc = launch_forward(c, d_in, B, &one, d_dets, d_counts, static_cast<hipStream_t>(stream));
  c->calib_raw = nullptr;
  return rc;
}

int ym_profile(ym_ctx* c, const float* d_in, int B, int H, int W, const ym_infer_args* args, float* d_dets,
               int* d_counts, void* stream, float* op_ms, int n_ops) {
  int rc = check_call(c, d_in, B, H, W, args, d_dets, d_counts);
  if (rc) return rc;
  if (!op_ms || n_ops < (int)c->ops.size()) return fail(YM_EINVAL, "op_ms must hold %zu entries", c->ops.size());
  HIPCK(hipSetDevice(c->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  if ((rc = ensure_workspace(c, B, H, W))) return rc;
  if ((rc = c->order_after_last(st))) return rc;
  const size_t ne = c->ops.size() + 1;
  while (c->prof_events.size() < ne) {
    hipEvent_t e;
    HIPCK(hipEventCreate(&e));
    c->prof_events.push_back(e);
  }
  // park the stream first so the host has queued every op + event before the GPU reaches them: the event pairs
  // then bracket device execution only (an eager host launch takes longer than most of these kernels)
  HIPCK(ym_launch_spin(20 * (int)c->ops.size() + 2000, st));
  HIPCK(hipEventRecord(c->prof_events[0], st));
  for (size_t i = 0; i < c->ops.size(); ++i) {
    if ((rc = launch_op(c, c->ops[i], B, d_in, args, d_dets, d_counts, st))) return rc;
    HIPCK(hipEventRecord(c->prof_events[i + 1], st));
  }
  HIPCK(hipEventSynchronize(c->prof_events[ne - 1]));
  for (size_t i = 0; i < c->ops.size(); ++i)
    HIPCK(hipEventElapsedTime(&op_ms[i], c->prof_events[i], c->prof_events[i + 1]));
  return YM_OK;
}

int ym_profile_replay(ym_ctx* c, const float* d_in, int B, int H, int W, const ym_infer_args* args, float* d_dets,
                      int* d_counts, void* stream, int reps, float* op_ms, int n_ops) {
  int rc = check_call(c, d_in, B, H, W, args, d_dets, d_counts);
  if (rc) return rc;
  if (!op_ms || n_ops < (int)c->ops.size()) return fail(YM_EINVAL, "op_ms must hold %zu entries", c->ops.size());
  if (reps < 1) reps = 20;
  HIPCK(hipSetDevice(c->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  if ((rc = ensure_workspace(c, B, H, W))) return rc;
  if ((rc = c->order_after_last(st))) return rc;
  // one real forward so every buffer holds this input's activations (and the /255 flag is set)
  for (const Op& op : c->ops)
    if ((rc = launch_op(c, op, B, d_in, args, d_dets, d_counts, st))) return rc;
  hipEvent_t e0, e1;
  HIPCK(hipEventCreate(&e0));
  HIPCK(hipEventCreate(&e1));
  for (size_t i = 0; i < c->ops.size(); ++i) {
    const Op& op = c->ops[i];
    const int k = op.r[0];
    op_ms[i] = -1.f;
    // input (resets counters), decode (appends candidates) and NMS (consumes them) are not idempotent: skipped
    if (k != OP_CONV && k != OP_DW && k != OP_SPPF && k != OP_ATTN) continue;
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    HIPCK(hipStreamBeginCapture(c->cap_stream, hipStreamCaptureModeRelaxed));
    int lrc = YM_OK;
    for (int r = 0; r < reps && lrc == YM_OK; ++r) lrc = launch_op(c, op, B, d_in, args, d_dets, d_counts, c->cap_stream);
    HIPCK(hipStreamEndCapture(c->cap_stream, &g));
    if (lrc != YM_OK) {
      (void)hipGraphDestroy(g);
      return lrc;
    }
    HIPCK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    HIPCK(hipGraphLaunch(ge, st));  // warm
    HIPCK(hipEventRecord(e0, st));
    HIPCK(hipGraphLaunch(ge, st));
    HIPCK(hipEventRecord(e1, st));
    HIPCK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCK(hipEventElapsedTime(&ms, e0, e1));
    op_ms[i] = ms / reps;
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return YM_OK;
}

int ym_tune(ym_ctx* c, const float* d_in, int B, int H, int W, const ym_infer_args* args, float* d_dets,
            int* d_counts, void* stream, int reps) {
  int rc = check_call(c, d_in, B, H, W, args, d_dets, d_counts);
  if (rc) return rc;
  HIPCK(hipSetDevice(c->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  if ((rc = ensure_workspace(c, B, H, W))) return rc;
  if ((rc = c->order_after_last(st))) return rc;
  if (reps < 1) reps = 8;
  // one real forward first so every buffer a candidate reads holds this model's activations
  c->drop_cfg(B, H, W);
  for (const Op& op : c->ops)
    if ((rc = launch_op(c, op, B, d_in, args, d_dets, d_counts, st))) return rc;
  HIPCK(hipStreamSynchronize(st));
  std::vector<int> best(c->ops.size(), -1);
  hipEvent_t e0, e1;
  HIPCK(hipEventCreate(&e0));
  HIPCK(hipEventCreate(&e1));
  const int ncfg = ym_conv_num_cfgs_dt(c->dtype);
  const char* tl = getenv("YM_TUNE_LOG");  // per-candidate timings to stderr (tools/)
  const bool tune_log = tl && *tl && *tl != '0';
  for (size_t i = 0; i < c->ops.size(); ++i) {
    const Op& op = c->ops[i];
    if (op.r[0] != OP_CONV) continue;
    ConvArgs a;
    int out_f32 = 0;
    if ((rc = conv_args(c, op, B, d_in, args->in_eps, a, out_f32))) return rc;
    if (a.nchw) continue;  // the stem has its own kernel (csrc/ym_stem.hip)
    // best config of one conv launch: time `reps` back-to-back launches of each candidate as one graph
    // (device-bound even for tiny kernels)
    auto tune_one = [&](const ConvArgs& ca, int of32, int& bcf) -> float {
      float bt = 1e30f;
      bcf = -1;
      for (int cf = 0; cf < ncfg; ++cf) {
        hipGraph_t g = nullptr;
        hipGraphExec_t ge = nullptr;
        HIPCK(hipStreamBeginCapture(c->cap_stream, hipStreamCaptureModeRelaxed));
        hipError_t le = hipSuccess;
        for (int r = 0; r < reps && le == hipSuccess; ++r) le = ym_launch_conv(c->dtype, of32, ca, cf, c->cap_stream, true);
        HIPCK(hipStreamEndCapture(c->cap_stream, &g));
        if (le != hipSuccess) {
          (void)hipGraphDestroy(g);
          continue;
        }
        HIPCK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        HIPCK(hipGraphLaunch(ge, st));
        HIPCK(hipEventRecord(e0, st));
        HIPCK(hipGraphLaunch(ge, st));
        HIPCK(hipGraphLaunch(ge, st));
        HIPCK(hipEventRecord(e1, st));
        HIPCK(hipEventSynchronize(e1));
        float ms = 0.f;
        HIPCK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(g);
        if (tune_log) fprintf(stderr, "[ym_tune] %s%s cfg %d: %.2f us\n", op.name, of32 < 0 ? "" : "", cf, ms * 1e3f / (2 * reps));
        if (ms < bt) { bt = ms; bcf = cf; }
      }
      return bt;
    };
    int cf = -1;
    const float tf = tune_one(a, out_f32, cf);
    best[i] = cf;
    if (a.w2) {  // fused pair: also the two convs as separate tuned launches
      ConvArgs A, Bc;
      split_args(c, op, a, A, Bc);
      int ca = -1, cb = -1;
      const float ta = tune_one(A, 0, ca), tb = tune_one(Bc, out_f32, cb);
      if (ca >= 0 && cb >= 0 && ta + tb < tf) best[i] = kSplitTag + 256 * ca + cb;
    }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  c->clear_graphs();
  c->put_cfg(B, H, W, best);
  return YM_OK;
}

int ym_get_op_cfg(ym_ctx* c, int B, int H, int W, int* cfg, int n) {
  if (!c || !cfg || n < (int)c->ops.size()) return fail(YM_EINVAL, "cfg array must hold %zu entries", c ? c->ops.size() : 0);
  const std::vector<int>* v = c->find_cfg(B, H, W);
  for (size_t i = 0; i < c->ops.size(); ++i) cfg[i] = (v && i < v->size()) ? (*v)[i] : -1;
  return v ? YM_OK : 1;
}

int ym_set_op_cfg(ym_ctx* c, int B, int H, int W, const int* cfg, int n) {
  if (!c || !cfg || n != (int)c->ops.size()) return fail(YM_EINVAL, "cfg array must hold %zu entries", c ? c->ops.size() : 0);
  for (int i = 0; i < n; ++i) {
    if (cfg[i] >= kSplitTag && c->ops[i].r[0] == OP_CONV && c->ops[i].r[30] &&
        ((cfg[i] - kSplitTag) >> 8) < ym_conv_num_cfgs_dt(c->dtype) &&
        ((cfg[i] - kSplitTag) & 255) < ym_conv_num_cfgs_dt(c->dtype))
      continue;  // a fused pair run as two launches
    if (cfg[i] >= ym_conv_num_cfgs_dt(c->dtype)) return fail(YM_EINVAL, "cfg[%d] = %d out of range", i, cfg[i]);
  }
  c->put_cfg(B, H, W, std::vector<int>(cfg, cfg + n));
  c->clear_graphs();
  return YM_OK;
}

int ym_num_ops(ym_ctx* c) { return c ? (int)c->ops.size() : fail(YM_EINVAL, "null context"); }

const char* ym_op_name(ym_ctx* c, int i) {
  if (!c || i < 0 || i >= (int)c->ops.size()) return "";
  return c->ops[i].name;
}

int ym_num_buffers(ym_ctx* c) { return c ? (int)c->bufs.size() : fail(YM_EINVAL, "null context"); }

int ym_buffer_info(ym_ctx* c, int b, void** ptr, int* C, int* H, int* W, int* elem_bytes) {
  if (!c || b < 0 || b >= (int)c->bufs.size()) return fail(YM_EINVAL, "bad buffer id");
  if (!c->d_arena) return fail(YM_ESTATE, "no workspace yet (run ym_infer first)");
  if (ptr) *ptr = c->bptr(b);
  if (C) *C = c->bufs[b].C;
  if (H) *H = c->buf_H(b);
  if (W) *W = c->buf_Wd(b);
  if (elem_bytes) *elem_bytes = c->elem(b);
  return YM_OK;
}

int ym_read_buffer(ym_ctx* c, int b, void* dst, size_t bytes) {
  if (!c || b < 0 || b >= (int)c->bufs.size() || !dst) return fail(YM_EINVAL, "bad buffer id or null dst");
  if (!c->d_arena) return fail(YM_ESTATE, "no workspace yet (run ym_infer first)");
  const size_t cap = (size_t)c->cB * c->buf_P(b) * c->bufs[b].C * c->elem(b);
  if (bytes > cap) return fail(YM_EINVAL, "read of %zu bytes exceeds buffer size %zu", bytes, cap);
  HIPCK(hipSetDevice(c->device));
  HIPCK(hipDeviceSynchronize());
  HIPCK(hipMemcpy(dst, c->bptr(b), bytes, hipMemcpyDefault));
  return YM_OK;
}

int ym_letterbox(ym_ctx* c, const void* d_src, int h, int w, int row_bytes, int bgr, int uh, int uw, int top,
                 int left, float* d_dst, int Hn, int Wn, void* stream) {
  if (!c) return fail(YM_EINVAL, "null context");
  if (!d_src || !d_dst || h < 1 || w < 1 || uh < 1 || uw < 1 || top < 0 || left < 0 || top + uh > Hn ||
      left + uw > Wn || row_bytes < 3 * w)
    return fail(YM_EINVAL, "bad ym_letterbox geometry (%dx%d -> %dx%d at (%d, %d) in %dx%d)", h, w, uh, uw, top, left,
                Hn, Wn);
  HIPCK(hipSetDevice(c->device));
  LetterboxArgs a{};
  a.src = static_cast<const unsigned char*>(d_src);
  a.h = h; a.w = w; a.row_bytes = row_bytes; a.bgr = bgr ? 1 : 0;
  a.uh = uh; a.uw = uw; a.top = top; a.left = left;
  a.scale_x = 1.0 / ((double)uw / w);  // cv2: scale_x = 1. / inv_scale_x, inv_scale_x = (double)dsize.width / ssize.width
  a.scale_y = 1.0 / ((double)uh / h);
  a.dst = d_dst; a.Hn = Hn; a.Wn = Wn;
  hipError_t e = ym_launch_letterbox(a, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return fail(YM_EHIP, "letterbox launch: %s", hipGetErrorString(e));
  return YM_OK;
}

static int launch_masks(ym_ctx* c, MaskArgs& a, int B, int H, int W, void* stream) {
  if (!c) return fail(YM_EINVAL, "null context");
  if (c->task != 1 || c->proto_buf < 0) return fail(YM_ESTATE, "ym_masks needs a segment plan");
  if (!c->d_arena || B > c->cB || H != c->cH || W != c->cW)
    return fail(YM_ESTATE, "ym_masks must follow ym_infer of the same (B, H, W) (workspace %dx%dx%d)", c->cB, c->cH,
                c->cW);
  HIPCK(hipSetDevice(c->device));
  a.proto = reinterpret_cast<const float*>(c->bptr(c->proto_buf));
  a.MH = c->buf_H(c->proto_buf); a.MW = c->buf_Wd(c->proto_buf); a.nm = c->nm;
  a.no = 6 + c->nm; a.B = B; a.H = H; a.W = W;
  if (a.total == 0) return YM_OK;
  if (!ym_masks_fused(a)) {  // the two-kernel path: (total, MH, MW) prototype-resolution scratch
    const size_t need = (size_t)a.total * a.MH * a.MW * sizeof(float);
    if (need > c->lowres_bytes) {
      if (c->d_lowres) HIPCK(hipFree(c->d_lowres));
      c->d_lowres = nullptr;
      hipError_t e = hipMalloc(&c->d_lowres, need);
      if (e != hipSuccess) return fail(YM_ENOMEM, "mask scratch hipMalloc(%zu): %s", need, hipGetErrorString(e));
      c->lowres_bytes = need;
    }
    a.lowres = c->d_lowres;
  }
  const hipError_t e = ym_launch_masks(a, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return fail(YM_EHIP, "mask kernels: %s", hipGetErrorString(e));
  return YM_OK;
}

int ym_masks(ym_ctx* c, const float* d_dets, int B, int max_det, const int* d_offsets, int total, int H, int W,
             unsigned char* d_masks, int* d_nonempty, void* stream) {
  if (total < 0 || max_det < 1 || (total > 0 && (!d_dets || !d_offsets || !d_masks || !d_nonempty)))
    return fail(YM_EINVAL, "bad ym_masks arguments");
  MaskArgs a{};
  a.dets = d_dets; a.max_det = max_det; a.offsets = d_offsets; a.total = total;
  a.masks = d_masks; a.nonempty = d_nonempty;
  return launch_masks(c, a, B, H, W, stream);
}

int ym_masks_slots(ym_ctx* c, const float* d_dets, int B, int max_det, const int* d_counts, int cap, int H, int W,
                   unsigned char* d_masks, int* d_flags, void* stream) {
  if (B < 1 || cap < 1 || max_det < 1 || cap > max_det || !d_dets || !d_counts || !d_masks || !d_flags)
    return fail(YM_EINVAL, "bad ym_masks_slots arguments");
  MaskArgs a{};
  a.dets = d_dets; a.max_det = max_det; a.counts = d_counts; a.cap = cap; a.total = B * cap;
  a.masks = d_masks; a.nonempty = d_flags;
  return launch_masks(c, a, B, H, W, stream);
}

// ---------------------------------------------------------------------------------------------- RCCL (xGMI)
// The init-time weight broadcast of the batch-sharded multi-GPU path: RCCL is resolved at run time
// (dlopen of the process's already-loaded librccl — torch's, when the host is Python — else the ROCm one), so
// libyolomi.so itself has no link-time dependency on it.  Only the four entry points below are used.
namespace {
struct Rccl {
  typedef int (*GetUniqueId)(void*);
  typedef int (*CommInitRank)(void**, int, ym_rccl_id, int);
  typedef int (*CommDestroy)(void*);
  typedef int (*CommUserRank)(void*, int*);
  typedef int (*CommCount)(void*, int*);
  typedef int (*Broadcast)(const void*, void*, size_t, int, int, void*, hipStream_t);
  typedef int (*AllReduce)(const void*, void*, size_t, int, int, void*, hipStream_t);
  typedef const char* (*ErrStr)(int);
  GetUniqueId get_id = nullptr;
  CommInitRank init = nullptr;
  CommDestroy destroy = nullptr;
  CommUserRank user_rank = nullptr;
  CommCount count = nullptr;
  Broadcast bcast = nullptr;
  AllReduce allreduce = nullptr;
  ErrStr err = nullptr;
  bool ok = false;
};

const Rccl* rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = nullptr;
    for (const char* n : {"librccl.so.1", "librccl.so"})
      if (!h) h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
    for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if (!h) h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
    if (!h) return x;
    x.get_id = (Rccl::GetUniqueId)dlsym(h, "ncclGetUniqueId");
    x.init = (Rccl::CommInitRank)dlsym(h, "ncclCommInitRank");
    x.destroy = (Rccl::CommDestroy)dlsym(h, "ncclCommDestroy");
    x.user_rank = (Rccl::CommUserRank)dlsym(h, "ncclCommUserRank");
    x.count = (Rccl::CommCount)dlsym(h, "ncclCommCount");
    x.bcast = (Rccl::Broadcast)dlsym(h, "ncclBroadcast");
    x.allreduce = (Rccl::AllReduce)dlsym(h, "ncclAllReduce");
    x.err = (Rccl::ErrStr)dlsym(h, "ncclGetErrorString");
    x.ok = x.get_id && x.init && x.destroy && x.user_rank && x.count && x.bcast && x.allreduce && x.err;
    return x;
  }();
  return r.ok ? &r : nullptr;
}

#define RCCLCK(x)                                                                                       \
  do {                                                                                                  \
    const int r_ = (x);                                                                                 \
    if (r_ != 0) return fail(YM_EHIP, "%s: RCCL error %d (%s)", #x, r_, R->err ? R->err(r_) : "?");     \
  } while (0)
constexpr int kNcclUint8 = 1, kNcclUint64 = 5;  // ncclDataType_t
constexpr int kNcclSum = 0;                       // ncclRedOp_t
constexpr size_t kBcastChunk = 16u << 20;         // blob bytes per broadcast (one staging buffer per rank)
}  // namespace

int ym_rccl_get_unique_id(ym_rccl_id* id) {
  if (!id) return fail(YM_EINVAL, "null id");
  const Rccl* R = rccl();
  if (!R) return fail(YM_ESTATE, "RCCL (librccl.so) is not available in this process");
  RCCLCK(R->get_id(id));
  return YM_OK;
}

int ym_rccl_comm_init(int device, int nranks, const ym_rccl_id* id, int rank, void** comm) {
  if (!id || !comm || nranks < 1 || rank < 0 || rank >= nranks) return fail(YM_EINVAL, "bad ym_rccl_comm_init arguments");
  const Rccl* R = rccl();
  if (!R) return fail(YM_ESTATE, "RCCL (librccl.so) is not available in this process");
  HIPCK(hipSetDevice(device));
  *comm = nullptr;
  RCCLCK(R->init(comm, nranks, *id, rank));
  return YM_OK;
}

int ym_rccl_comm_destroy(void* comm) {
  if (!comm) return YM_OK;
  const Rccl* R = rccl();
  if (!R) return fail(YM_ESTATE, "RCCL (librccl.so) is not available in this process");
  RCCLCK(R->destroy(comm));
  return YM_OK;
}

// ---- the init-time weight broadcast: one rank's side, shared by the two transports
// (ym_broadcast_weights: RCCL, one rank per process; ym_broadcast_weights_local: every rank's context in this process,
// the fake backend of SURVEY §4.4) — staging buffer, the root's upload, a receiver's copy-out and load, and the
// verdict every rank agrees on.  The transports only move the chunk between staging buffers and sum control words.
struct BcastRank {
  ym_ctx* c = nullptr;
  int rank = -1;
  bool hip_ok = true, copy_ok = true;
  char* d = nullptr;  // kBcastChunk staging bytes on the context's device
  std::vector<char> h;  // a receiver's copy of the blob
  int rc = YM_OK;
  BcastRank() = default;
  BcastRank(const BcastRank&) = delete;
  BcastRank& operator=(const BcastRank&) = delete;
  ~BcastRank() {
    if (d) (void)hipFree(d);
  }
  // step (1): this rank's contribution to {the root's blob size (0: the root has no weights), staging failures}
  void open(int root, unsigned long long h1[2]) {
    hip_ok = hipSetDevice(c->device) == hipSuccess;
    const bool alloc_ok = hip_ok && hipMalloc(&d, kBcastChunk) == hipSuccess;
    if (!alloc_ok) d = nullptr;
    h1[0] += (rank == root && c->loaded) ? (unsigned long long)c->blob_host.size() : 0ull;
    h1[1] += alloc_ok ? 0ull : 1ull;
    copy_ok = hip_ok;
  }
  // step (2), per chunk: the root uploads it into its staging buffer before the transport moves it ...
  void put(int root, unsigned long long off, size_t len, hipStream_t st) {
    if (rank == root)
      copy_ok = copy_ok && hipMemcpyAsync(d, c->blob_host.data() + off, len, hipMemcpyHostToDevice, st) == hipSuccess;
  }
  // ... and a receiver copies it out after (the staging buffer is reused by the next chunk)
  void get(int root, unsigned long long off, size_t len, hipStream_t st) {
    if (rank != root)
      copy_ok = copy_ok && hipMemcpyAsync(h.data() + off, d, len, hipMemcpyDeviceToHost, st) == hipSuccess;
    copy_ok = copy_ok && hipStreamSynchronize(st) == hipSuccess;
  }
  // step (3): a receiver loads what it got; returns this rank's failure count for the verdict all-reduce
  unsigned long long load(int root, unsigned long long nbytes) {
    rc = copy_ok ? YM_OK : fail(YM_EHIP, "blob staging copy failed");
    if (rc == YM_OK && rank != root) rc = ym_load_weights(c, h.data(), nbytes);
    return rc == YM_OK ? 0ull : 1ull;
  }
};

// The identical-on-every-rank verdict on step (1)'s sums: YM_OK or the error every rank returns before step (2).
static int bcast_check(const unsigned long long h1[2], bool is_root, int root) {
  if (h1[0] == 0)
    return fail(YM_ESTATE, is_root ? "the root context has no weights to broadcast"
                                   : "the root rank %d has no weights to broadcast", root);
  if (h1[0] < kHdr * 4 || h1[0] > (1ull << 34)) return fail(YM_EBLOB, "broadcast blob size %llu", h1[0]);
  if (h1[1]) return fail(YM_ENOMEM, "%llu rank(s) could not allocate the %zu-byte staging buffer", h1[1], kBcastChunk);
  return YM_OK;
}

// The root rank's loaded blob (plan + weights, exactly the bytes its ym_load_weights received) goes to every rank
// of `comm` over RCCL (xGMI) and each non-root rank loads it into `c` (ym_load_weights), so every rank ends with an
// identical model without touching the file system.  Synchronous.
// Every rank issues the same sequence of collectives whatever fails locally, so no rank is left waiting inside RCCL
// for one that returned early: (1) an all-reduce (sum) of {root's blob size (0: the root has no weights), ranks
// whose staging buffer failed to allocate}; only if both are valid, (2) the blob broadcast in kBcastChunk pieces
// and (3) an all-reduce of the per-rank copy / load failures, so every rank returns the same verdict.  Errors in the
// arguments themselves (null pointers, root out of range) are identical on every rank and return before any
// collective; an RCCL error is communicator-wide.
int ym_broadcast_weights(ym_ctx* c, void* comm, int root, void* stream) {
  if (!c || !comm) return fail(YM_EINVAL, "null argument");
  const Rccl* R = rccl();
  if (!R) return fail(YM_ESTATE, "RCCL (librccl.so) is not available in this process");
  int rank = -1, n = 0;
  RCCLCK(R->user_rank(comm, &rank));
  RCCLCK(R->count(comm, &n));
  if (root < 0 || root >= n) return fail(YM_EINVAL, "root %d out of range (%d ranks)", root, n);
  const hipStream_t st = static_cast<hipStream_t>(stream);
  BcastRank me;
  me.c = c;
  me.rank = rank;
  // control words: the context's 4 KB scratch (allocated by ym_create, so nothing can fail before step 1)
  unsigned long long* dctl = reinterpret_cast<unsigned long long*>(c->d_misc + 8192);
  auto allreduce_sum = [&](unsigned long long* h, int cnt) -> int {
    me.hip_ok = me.hip_ok && hipMemcpyAsync(dctl, h, 8 * cnt, hipMemcpyHostToDevice, st) == hipSuccess;
    const int r = R->allreduce(dctl, dctl, cnt, kNcclUint64, kNcclSum, comm, st);
    if (r) return r;
    me.hip_ok = me.hip_ok && hipMemcpyAsync(h, dctl, 8 * cnt, hipMemcpyDeviceToHost, st) == hipSuccess &&
                hipStreamSynchronize(st) == hipSuccess;
    return 0;
  };
  unsigned long long h1[2] = {0ull, 0ull};
  me.open(root, h1);
  int r = allreduce_sum(h1, 2);  // (1)
  if (r) return fail(YM_EHIP, "ncclAllReduce(size): %s", R->err(r));
  if (int e = bcast_check(h1, rank == root, root)) return e;
  const unsigned long long nbytes = h1[0];
  if (rank != root) me.h.resize(nbytes);
  for (unsigned long long off = 0; off < nbytes; off += kBcastChunk) {  // (2)
    const size_t len = (size_t)std::min<unsigned long long>(kBcastChunk, nbytes - off);
    me.put(root, off, len, st);
    r = R->bcast(me.d, me.d, len, kNcclUint8, root, comm, st);
    if (r) return fail(YM_EHIP, "ncclBroadcast(blob): %s", R->err(r));
    me.get(root, off, len, st);
  }
  unsigned long long h3[1] = {me.load(root, nbytes)};  // (3)
  r = allreduce_sum(h3, 1);
  if (r) return fail(YM_EHIP, "ncclAllReduce(status): %s", R->err(r));
  if (me.rc != YM_OK) return me.rc;
  if (h3[0]) return fail(YM_EBLOB, "the weight broadcast failed on %llu other rank(s)", h3[0]);
  return YM_OK;
}

// The fake backend of the same broadcast (N ranks as N contexts of this process, e.g. on one GPU):
// rank i is ctxs[i]; the all-reduces are host sums and the chunk moves from the root's staging buffer to every
// other rank's by a device-to-device copy on `stream`, between the same BcastRank put / get / load steps the RCCL
// transport runs.  Returns the status of the first failing rank (every rank's context is left loaded or not as in
// the RCCL path); on success every context holds the root's blob.
int ym_broadcast_weights_local(ym_ctx* const* ctxs, int n, int root, void* stream) {
  if (!ctxs || n < 1) return fail(YM_EINVAL, "null / empty context list");
  if (root < 0 || root >= n) return fail(YM_EINVAL, "root %d out of range (%d ranks)", root, n);
  for (int i = 0; i < n; ++i)
    if (!ctxs[i]) return fail(YM_EINVAL, "null context for rank %d", i);
  const hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<BcastRank> ranks(n);
  unsigned long long h1[2] = {0ull, 0ull};
  for (int i = 0; i < n; ++i) {  // (1)
    ranks[i].c = ctxs[i];
    ranks[i].rank = i;
    ranks[i].open(root, h1);
  }
  if (int e = bcast_check(h1, true, root)) return e;
  const unsigned long long nbytes = h1[0];
  for (int i = 0; i < n; ++i)
    if (i != root) ranks[i].h.resize(nbytes);
  for (unsigned long long off = 0; off < nbytes; off += kBcastChunk) {  // (2)
    const size_t len = (size_t)std::min<unsigned long long>(kBcastChunk, nbytes - off);
    ranks[root].put(root, off, len, st);
    for (int i = 0; i < n; ++i)
      if (i != root)
        ranks[i].copy_ok = ranks[i].copy_ok && ranks[root].copy_ok &&
                           hipMemcpyAsync(ranks[i].d, ranks[root].d, len, hipMemcpyDeviceToDevice, st) == hipSuccess;
    for (int i = 0; i < n; ++i) ranks[i].get(root, off, len, st);
  }
  unsigned long long h3 = 0;  // (3)
  for (int i = 0; i < n; ++i) h3 += ranks[i].load(root, nbytes);
  for (int i = 0; i < n; ++i)
    if (ranks[i].rc != YM_OK) return ranks[i].rc;
  return h3 ? fail(YM_EBLOB, "the weight broadcast failed on %llu rank(s)", h3) : YM_OK;
}

int ym_sync(ym_ctx* c) {
  if (!c) return fail(YM_EINVAL, "null context");
  HIPCK(hipSetDevice(c->device));
  HIPCK(hipDeviceSynchronize());
  return YM_OK;
}

void ym_destroy(ym_ctx* c) { delete c; }

}  // extern "C"
