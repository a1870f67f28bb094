// ggml-hip-fuse.cpp — the hook path's node scheduler: held-node snapshots, launch fusion of the chains
// ggml emits back to back, sibling q4_0 GEMV groups and the elementwise batches they hold.
#include "ggml-hip-internal.h"

using namespace ghh;

namespace ghh {

// ------------------------------------------------------------------------------------------
// Launch fusion of back-to-back full-offload nodes.  A decode token is ~830 dependent launches of
// ~2.6 us host cost each (tools/host_costs.hip), so chains that ggml emits one after the other are
// run as one kernel: add -> rms_norm -> mul(norm weight), rms_norm -> mul, scale -> diag_mask_inf
// -> soft_max, silu ... mul (across the one q4_0 mul_mat between them), rope -> cpy (into the K
// cache) and the f16 mul_mat KQV -> permute(0,2,1,3) -> contiguous cpy.  The producer node is
// deferred until its consumer arrives; anything else flushes it first, and so does every other
// backend entry point (its output is device memory, observable only through the backend).  The
// fused kernels store every intermediate tensor as its own node would, bit for bit.
// GGML_HIP_FUSE=0 runs every node as its own launch.

// GGML_HIP_NORM_FOLD: 1 (default) the decode norm chains and silu -> mul run in the consuming GEMVs' x
// prologue, 2 the norm chains only, 0 neither (each chain its own launch)
std::atomic<int> g_norm_fold{-1};
int norm_fold_mode() {
    int v = g_norm_fold.load(std::memory_order_relaxed);
    if (v < 0) {
        v = getenv("GGML_HIP_NORM_FOLD") ? atoi(getenv("GGML_HIP_NORM_FOLD")) : 1;
        v = v < 0 || v > 2 ? 1 : v;
        g_norm_fold.store(v, std::memory_order_relaxed);
    }
    return v;
}
bool norm_fold_enabled() { return norm_fold_mode() != 0; }
bool silu_fold_enabled() { return norm_fold_mode() == 1; }

// GGML_HIP_X9_FOLD=0: a prefill norm / silu chain whose consumers all take k_gemm9 runs as its own
// launch and the mul_mats build the x image themselves (k_prep9_x); on (default), the chain's kernel
// writes the image beside its f32 output
std::atomic<int> g_x9_fold{-1};
bool x9_fold_enabled() {
    int v = g_x9_fold.load(std::memory_order_relaxed);
    if (v < 0) {
        v = (!getenv("GGML_HIP_X9_FOLD") || atoi(getenv("GGML_HIP_X9_FOLD")) != 0) ? 1 : 0;
        g_x9_fold.store(v, std::memory_order_relaxed);
    }
    return v == 1;
}

// GGML_HIP_GEMV_EPI=0: the elementwise nodes held behind a decode q|k|v norm group (rope K -> K cache,
// V -> V cache, rope Q) run as their own batched launch; on (default), in the GEMV's epilogue
std::atomic<int> g_epi_fold{-1};
bool epi_fold_enabled() {
    int v = g_epi_fold.load(std::memory_order_relaxed);
    if (v < 0) {
        v = (!getenv("GGML_HIP_GEMV_EPI") || atoi(getenv("GGML_HIP_GEMV_EPI")) != 0) ? 1 : 0;
        g_epi_fold.store(v, std::memory_order_relaxed);
    }
    return v == 1;
}

// GGML_HIP_KQ_FOLD=0: the decode KQ runs as its own launch before the soft_max -> KQV chain; on (default)
// the chain's launch computes it
std::atomic<int> g_kq_fold{-1};
bool kq_fold_enabled() {
    int v = g_kq_fold.load(std::memory_order_relaxed);
    if (v < 0) {
        v = (!getenv("GGML_HIP_KQ_FOLD") || atoi(getenv("GGML_HIP_KQ_FOLD")) != 0) ? 1 : 0;
        g_kq_fold.store(v, std::memory_order_relaxed);
    }
    return v == 1;
}

std::atomic<int> g_fuse{-1};
bool fuse_enabled() {
    int v = g_fuse.load(std::memory_order_relaxed);
    if (v < 0) {
        v = (!getenv("GGML_HIP_FUSE") || atoi(getenv("GGML_HIP_FUSE")) != 0) ? 1 : 0;
        g_fuse.store(v, std::memory_order_relaxed);
    }
    return v == 1;
}

// ---- held-node snapshots (graph lifetime).  A held node (pending chain, group member, node held
// behind a group) can outlive its ggml_graph_compute: a caller may end a graph on a device-only node
// and ggml_free the context before the next backend call flushes it.  Every node is therefore copied
// when it is held, with its operands two levels deep, into a backend-owned arena; the copies carry
// everything a deferred launch reads (shapes, strides, extras, the host scalar parameters of scale /
// rope / diag_mask_inf), and flushes run on the copies only.  Identity tests against an arriving
// node (t->src0 == held) compare the original address AND the original's fields at hold time, so a
// new graph that reuses a freed address never fuses with a stale node.
struct SnapTensor {
    tensor t;                  // working copy: src0 / src1 -> copies, host parameters -> param
    const tensor *orig = nullptr;
    tensor pristine;           // the original's bytes when it was copied
    int depth = -1;
    alignas(16) uint8_t param[16];
};
constexpr size_t SNAP_BLOCK = 1024;
struct SnapArena {
    std::vector<std::unique_ptr<SnapTensor[]>> blocks;     // stable addresses
    size_t used = 0;
    std::unordered_map<const tensor *, SnapTensor *> memo;  // original -> copy
};
SnapArena g_snaps;

bool is_snap(const tensor *t) {
    for (const auto &b : g_snaps.blocks)
        if ((const char *)t >= (const char *)b.get() && (const char *)t < (const char *)(b.get() + SNAP_BLOCK)) return true;
    return false;
}
// the fields a graph does not change after building it (n_tasks and the perf counters excluded)
bool stable_equal(const tensor *a, const tensor *b) {
    return memcmp(a, b, offsetof(tensor, n_tasks)) == 0 &&
           memcmp(&a->data, &b->data, offsetof(tensor, padding) - offsetof(tensor, data)) == 0;
}
tensor *snap(tensor *t, int depth) {
    if (!t || is_snap(t)) return t;
    auto it = g_snaps.memo.find(t);
    SnapTensor *c = nullptr;
    if (it != g_snaps.memo.end() && stable_equal(t, &it->second->pristine)) {
        c = it->second;
        if (c->depth >= depth) return &c->t;
    } else {                   // new, or a freed address reused by another tensor: a fresh copy
        const size_t bi = g_snaps.used / SNAP_BLOCK;
        if (bi == g_snaps.blocks.size()) g_snaps.blocks.emplace_back(new SnapTensor[SNAP_BLOCK]);
        c = &g_snaps.blocks[bi][g_snaps.used % SNAP_BLOCK];
        g_snaps.used++;
        c->t = *t;
        c->pristine = *t;
        c->orig = t;
        c->t.grad = nullptr;
        for (int i = 0; i < gabi::MAX_OPT; i++) c->t.opt[i] = nullptr;
        c->t.src0 = c->t.src1 = nullptr;
        if (t->backend == gabi::BACKEND_CPU && t->data && (t->type == gabi::TYPE_F32 || t->type == gabi::TYPE_I32) &&
            gabi::nbytes(t) <= sizeof(c->param)) {
            memcpy(c->param, t->data, gabi::nbytes(t));
            c->t.data = c->param;
        }
        g_snaps.memo[t] = c;
    }
    c->depth = depth;
    if (depth > 0) {           // t is the live original here: it is being held right now
        c->t.src0 = snap(t->src0, depth - 1);
        c->t.src1 = snap(t->src1, depth - 1);
    }
    return &c->t;
}
tensor *hold(tensor *t) { return snap(t, 2); }
void snap_reset() {
    g_snaps.used = 0;
    g_snaps.memo.clear();
}
// is x (arriving, or a copy) the tensor h (a held copy)?
bool same_tensor(const tensor *x, const tensor *h) {
    if (x == h) return true;
    if (!x || !h) return false;
    const bool sx = is_snap(x), sh = is_snap(h);
    if (sx == sh) return false;            // two copies (one per tensor) or two live originals
    const SnapTensor *c = (const SnapTensor *)(sh ? h : x);
    const tensor *o = sh ? x : h;
    return o == c->orig && stable_equal(o, &c->pristine);
}

struct Pending {
    int n = 0;
    tensor *node[4] = {};
};
Pending g_pend;
// The decode KQ (f16 K view . f32 q, one query row per head), held for the scale -> diag_mask_inf ->
// soft_max -> KQV -> merge chain that follows it: the chain's launch computes it first (op_kq_softmax_kqv).
// Run on its own (run_device_op) when anything else comes first.
tensor *g_kq = nullptr;
void flush_kq() {
    tensor *t = g_kq;
    g_kq = nullptr;
    if (t) run_device_op(t);
}

// ---- a completed chain of one row (decode) that produces the src1 of q4_0 mul_mats, held for them:
// they run it in their x prologue (ghip::gemv_q4_0_multi_norm), one launch less per chain; anything
// else runs it as its own launch.  kind 1: [add ->] rms_norm -> mul (op_add_rms_norm_mul_f32; out =
// the mul), kind 2: silu -> mul (op_silu_mul_f32; a = the silu input, b = the mul's other operand,
// norm = the silu output)
struct NormChain {
    bool on = false;
    int kind = 1;
    int nn = 0;
    tensor *node[3] = {};          // held copies of the chain's nodes (for the counters)
    tensor *out_node = nullptr;    // the chain's last node (its output is the GEMVs' src1)
    const float *a = nullptr, *b = nullptr, *w = nullptr;
    float *sum = nullptr, *norm = nullptr, *out = nullptr;
    const uint16_t *table = nullptr;
    int64_t ncols = 0;
    int64_t nrows = 1;             // > 1: a prefill chain held for q4_0 mul_mats on fp6 images (x image fold)
};
NormChain g_norm;
void mul_mat_node(const tensor *src0, const tensor *src1, tensor *dst);

char *dptr(const tensor *t) { return (char *)((ggml_tensor_extra_gpu *)t->extra)->data_device[g_main_device]; }
bool dev_f32(const tensor *t) {
    return t && t->backend == gabi::BACKEND_GPU && t->type == gabi::TYPE_F32 && t->extra && is_contiguous(t);
}
bool host_scalar_param(const tensor *t) { return t && t->backend == gabi::BACKEND_CPU && t->data; }
bool overlaps(const tensor *a, const tensor *b) {   // device byte ranges of two device tensors
    if (!a || !b || a->backend != gabi::BACKEND_GPU || b->backend != gabi::BACKEND_GPU || !a->extra || !b->extra) return false;
    const char *pa = dptr(a), *pb = dptr(b);
    return pa < pb + gabi::nbytes(b) && pb < pa + gabi::nbytes(a);
}

bool deferrable(const tensor *t) {
    if (!fuse_enabled() || !dev_f32(t)) return false;
    switch (t->op) {
        case gabi::OP_ADD:
            return dev_f32(t->src0) && dev_f32(t->src1) && same_shape(t, t->src0) && same_shape(t, t->src1);
        case gabi::OP_RMS_NORM:
        case gabi::OP_SILU:
            return dev_f32(t->src0) && same_shape(t, t->src0);
        case gabi::OP_SCALE:
            return dev_f32(t->src0) && same_shape(t, t->src0) && host_scalar_param(t->src1);
        case gabi::OP_ROPE:
            return dev_f32(t->src0) && same_shape(t, t->src0) && t->ne[3] == 1 && host_scalar_param(t->src1) &&
                   ((const int32_t *)t->src1->data)[2] == 0;
        case gabi::OP_MUL_MAT:       // f16 x f32 (attention): the consumer may be the KQV merge copy
            return t->src0 && t->src0->type == gabi::TYPE_F16 && t->src0->backend == gabi::BACKEND_GPU && t->src1 &&
                   t->src1->type == gabi::TYPE_F32 && t->src1->backend == gabi::BACKEND_GPU && t->src1->extra;
        default:
            return false;
    }
}

void count_node(const tensor *t) { g_op_count[t->op].fetch_add(1, std::memory_order_relaxed); }

// the pending scale -> diag_mask_inf -> soft_max chain (nodes 0..2 of p) in one launch
void launch_softmax_chain(const Pending &p) {
    const tensor *sc = p.node[0], *mk = p.node[1], *t = p.node[2];
    const int id = g_main_device;
    hipStream_t s = g_dev[id].stream;
    const OpTables &tb = op_tables(id, s);
    float *d = (float *)dptr(t);
    HIP_FATAL(hipSetDevice(id));
    HIP_FATAL(ghip::op_scale_mask_soft_max_f32((const float *)dptr(sc->src0), dptr(sc) == (char *)d ? nullptr : (float *)dptr(sc),
                                               dptr(mk) == (char *)d ? nullptr : (float *)dptr(mk), d,
                                               *(const float *)sc->src1->data, t->ne[0], gabi::nrows(t), t->ne[1],
                                               ((const int32_t *)mk->src1->data)[0], tb.exp, s));
    for (int i = 0; i < 3; i++) count_node(p.node[i]);
    g_fused[1].fetch_add(1, std::memory_order_relaxed);
}
bool softmax_chain(const Pending &p) {
    return p.n >= 3 && p.node[0]->op == gabi::OP_SCALE && p.node[1]->op == gabi::OP_DIAG_MASK_INF &&
           p.node[2]->op == gabi::OP_SOFT_MAX;
}

void flush_pending() {
    flush_kq();                         // the chain reads its output
    const Pending p = g_pend;
    g_pend = Pending{};
    int i = 0;
    if (softmax_chain(p)) {             // held lazily for a possible KQV: complete it as one launch
        launch_softmax_chain(p);
        i = 3;
    }
    for (; i < p.n; i++) run_device_op(p.node[i]);
}

bool dev_overlap(const tensor *a, const tensor *b);
size_t span_bytes(const tensor *t);

// a chain of nrows rows that may be held for the k_gemm9 x image fold
bool x9_chain_ok(int64_t ncols, int64_t nrows) {
    return x9_fold_enabled() && !exact_mode() && gemm_version() == 10 && nrows > IMG_MIN_N && ghip::op_x9_ok(ncols, nrows) &&
           nrows * ncols < ((int64_t)1 << 31);
}

// a decode KQ that op_kq_softmax_kqv can compute: K (f16, element stride 2) and q (f32, contiguous head
// rows) on the device, one query row per head, head dimension <= 256, a contiguous [nkv][1][heads] output
bool kq_holdable(const tensor *t) {
    if (!fuse_enabled() || !kq_fold_enabled() || t->op != gabi::OP_MUL_MAT || !dev_f32(t)) return false;
    const tensor *K = t->src0, *Q = t->src1;
    return K && Q && K->type == gabi::TYPE_F16 && K->backend == gabi::BACKEND_GPU && K->extra && Q->type == gabi::TYPE_F32 &&
           Q->backend == gabi::BACKEND_GPU && Q->extra && K->nb[0] == 2 && Q->nb[0] == 4 && K->ne[3] == 1 && Q->ne[3] == 1 &&
           Q->ne[1] == 1 && K->ne[0] == Q->ne[0] && K->ne[0] >= 1 && K->ne[0] <= 256 && K->ne[2] == Q->ne[2] &&
           t->ne[0] == K->ne[1] && t->ne[1] == 1 && t->ne[2] == K->ne[2] && t->ne[3] == 1 && (Q->nb[2] & 3) == 0;
}
// ... whose output the held soft_max chain reads row for row (sm: the chain's soft_max node), for rows up to
// GGML_HIP_KQ_FOLD_MAX keys (default 192): each of a head's workgroups computes the whole KQ row, so past a
// few hundred keys KQ's own launch over every CU is faster (tools/attn_ab.py: 7.3 vs 7.5 us at 136 keys,
// 8.3 vs 7.6 at 256, 12.2 vs 9.3 at 512)
bool kq_chain_ok(const tensor *kqn, const tensor *sm) {
    static const int64_t max_kv = getenv("GGML_HIP_KQ_FOLD_MAX") ? atoll(getenv("GGML_HIP_KQ_FOLD_MAX")) : 192;
    return sm->ne[0] == kqn->ne[0] && sm->ne[1] == 1 && sm->ne[2] == kqn->ne[2] && kqn->ne[0] <= max_kv;
}

// t arrives while a chain is pending: extend the chain, complete it in one launch, or let a q4_0
// mul_mat that touches none of its buffers run first.  false: t does not fit (caller flushes).
bool try_fuse(tensor *t) {
    Pending &p = g_pend;
    tensor *last = p.node[p.n - 1];
    const int id = g_main_device;
    hipStream_t s = g_dev[id].stream;
    // add -> rms_norm(sum): extend
    if (p.n == 1 && last->op == gabi::OP_ADD && t->op == gabi::OP_RMS_NORM && same_tensor(t->src0, last) && deferrable(t)) {
        p.node[p.n++] = hold(t);
        return true;
    }
    // scale -> diag_mask_inf(scaled): extend
    if (p.n == 1 && last->op == gabi::OP_SCALE && t->op == gabi::OP_DIAG_MASK_INF && same_tensor(t->src0, last) && dev_f32(t) &&
        same_shape(t, last) && host_scalar_param(t->src1)) {
        p.node[p.n++] = hold(t);
        return true;
    }
    // [add ->] rms_norm -> mul(norm weight row): complete
    if (last->op == gabi::OP_RMS_NORM && t->op == gabi::OP_MUL && same_tensor(t->src0, last) && dev_f32(t) && same_shape(t, last) &&
        dev_f32(t->src1) && t->src1->ne[0] == t->ne[0] && t->src1->ne[1] == 1 && t->src1->ne[2] == 1 && t->src1->ne[3] == 1) {
        const tensor *add = p.n == 2 ? p.node[0] : nullptr;
        const tensor *x = add ? add : last->src0;     // the rms_norm input
        // one row (decode): hold it for the q4_0 GEMVs that follow (norm_fold)
        NormChain c;
        c.a = add ? (const float *)dptr(add->src0) : nullptr;
        c.b = add ? (const float *)dptr(add->src1) : (const float *)dptr(x);
        c.sum = add ? (float *)dptr(add) : nullptr;
        c.norm = (float *)dptr(last);
        c.w = (const float *)dptr(t->src1);
        c.out = (float *)dptr(t);
        c.ncols = t->ne[0];
        auto al = [](const void *q) { return ((uintptr_t)q & 15) == 0; };
        bool fold = norm_fold_enabled() && !exact_mode() && gabi::nrows(t) == 1 && c.ncols % 64 == 0 &&
                    c.ncols <= 16384 && al(c.a) && al(c.b) && al(c.sum) && al(c.norm) && al(c.w) && al(c.out);
        // the chain's outputs must not alias its inputs (the GEMV's workgroups read the inputs while
        // workgroup 0 stores the outputs)
        for (const tensor *o : {add, (const tensor *)last, (const tensor *)t})
            for (const tensor *i : {(const tensor *)(add ? add->src0 : nullptr), (const tensor *)(add ? add->src1 : x),
                                    (const tensor *)t->src1})
                if (o && i && dev_overlap(o, i)) fold = false;
        // many rows (prefill): hold it too; if the q4_0 mul_mats that consume it all take k_gemm9, its
        // launch writes their x image (flush_group_x9), else it runs as below when they flush it
        if (x9_chain_ok(c.ncols, gabi::nrows(t)) && al(c.a) && al(c.b) && al(c.sum) && al(c.norm) && al(c.w) && al(c.out)) {
            fold = true;
            c.nrows = gabi::nrows(t);
        }
        if (fold) {
            for (int i = 0; i < p.n; i++) c.node[c.nn++] = p.node[i];
            c.node[c.nn++] = hold(t);
            c.out_node = c.node[c.nn - 1];
            c.on = true;
            g_norm = c;
            p = Pending{};
            return true;
        }
        HIP_FATAL(hipSetDevice(id));
        HIP_FATAL(ghip::op_add_rms_norm_mul_f32(add ? (const float *)dptr(add->src0) : nullptr,
                                                add ? (const float *)dptr(add->src1) : (const float *)dptr(x),
                                                add ? (float *)dptr(add) : nullptr, (float *)dptr(last),
                                                (const float *)dptr(t->src1), (float *)dptr(t), t->ne[0], gabi::nrows(t), s));
        for (int i = 0; i < p.n; i++) count_node(p.node[i]);
        count_node(t);
        g_fused[0].fetch_add(1, std::memory_order_relaxed);
        p = Pending{};
        return true;
    }
    // scale -> diag_mask_inf -> soft_max: held (completed as one launch by flush_pending, or with
    // the KQV that follows at decode)
    if (p.n == 2 && p.node[0]->op == gabi::OP_SCALE && last->op == gabi::OP_DIAG_MASK_INF && t->op == gabi::OP_SOFT_MAX &&
        same_tensor(t->src0, last) && dev_f32(t) && same_shape(t, last)) {
        p.node[p.n++] = hold(t);
        return true;
    }
    // soft_max chain -> KQV (f16 V^T . softmax, one query row per head): extend
    if (p.n == 3 && softmax_chain(p) && t->op == gabi::OP_MUL_MAT && same_tensor(t->src1, last) && t->src0 &&
        t->src0->type == gabi::TYPE_F16 && t->src0->backend == gabi::BACKEND_GPU && t->src0->extra &&
        t->src0->nb[0] == 2 && t->src0->ne[3] == 1 && last->ne[1] == 1 && last->ne[3] == 1 &&
        t->src0->ne[0] == last->ne[0] && t->src0->ne[2] == last->ne[2] && last->ne[0] <= 16384 && dev_f32(t) &&
        t->ne[1] == 1 && t->ne[0] == t->src0->ne[1] && dev_f32(p.node[0]->src0)) {
        p.node[p.n++] = hold(t);
        return true;
    }
    // soft_max chain -> KQV -> cpy(permute(KQV)) (the merged heads): complete as one launch
    if (p.n == 4 && softmax_chain(p) && t->op == gabi::OP_CPY && t->src0 && t->src0->op == gabi::OP_PERMUTE &&
        same_tensor(t->src0->src0, last)) {
        const tensor *m = t->src0, *cb = t->src1;
        if (m->ne[0] == last->ne[0] && m->ne[1] == last->ne[2] && m->ne[2] == last->ne[1] && m->ne[3] == 1 &&
            m->nb[0] == 4 && m->nb[1] == last->nb[2] && m->nb[2] == last->nb[1] && dev_f32(cb) &&
            gabi::nbytes(cb) == gabi::nbytes(last) && !overlaps(cb, last) && !overlaps(cb, last->src0) &&
            !overlaps(cb, p.node[2]) && !overlaps(cb, p.node[0]->src0)) {
            const tensor *sc = p.node[0], *mk = p.node[1], *sm = p.node[2], *kqv = last, *vv = kqv->src0;
            const char *kq = dptr(sc->src0);
            // stores into the buffer the workgroups read (the in-place chain) are skipped: see
            // k_softmax_kqv; no node reads them, KQV consumes the softmax inside the launch
            auto out = [&](const tensor *x) { return overlaps(x, sc->src0) ? nullptr : (float *)dptr(x); };
            const OpTables &tb = op_tables(id, s);
            HIP_FATAL(hipSetDevice(id));
            tensor *kqn = g_kq;
            if (kqn && same_tensor(sc->src0, kqn) && kq_chain_ok(kqn, sm)) {
                // KQ in the same launch: no workgroup reads kq from memory, so every buffer of the chain is
                // stored once, by the last tensor of the chain that owns it (in-place scale / mask / soft_max)
                const tensor *chain[4] = {kqn, sc, mk, sm};
                float *st[4];
                for (int i = 0; i < 4; i++) {
                    st[i] = (float *)dptr(chain[i]);
                    for (int k = i + 1; k < 4; k++)
                        if (dev_overlap(chain[i], chain[k])) st[i] = nullptr;
                }
                const tensor *K = kqn->src0, *Q = kqn->src1;
                g_kq = nullptr;
                HIP_FATAL(ghip::op_kq_softmax_kqv(dptr(K), K->nb[1], K->nb[2], (const float *)dptr(Q), Q->nb[2], (int)K->ne[0],
                                                  st[0], st[1], st[2], st[3], *(const float *)sc->src1->data,
                                                  ((const int32_t *)mk->src1->data)[0], tb.exp, sm->ne[0], sm->ne[2], dptr(vv),
                                                  vv->nb[1], vv->nb[2], vv->ne[1], (float *)dptr(kqv), (float *)dptr(cb), s));
                count_node(kqn);
                g_fused[14].fetch_add(1, std::memory_order_relaxed);
            } else {
                flush_kq();
                HIP_FATAL(ghip::op_softmax_kqv((const float *)kq, out(sc), out(mk), out(sm), *(const float *)sc->src1->data,
                                               ((const int32_t *)mk->src1->data)[0], tb.exp, sm->ne[0], sm->ne[2], dptr(vv),
                                               vv->nb[1], vv->nb[2], vv->ne[1], (float *)dptr(kqv), (float *)dptr(cb), s));
            }
            for (int i = 0; i < p.n; i++) count_node(p.node[i]);
            count_node(t);
            g_fused[8].fetch_add(1, std::memory_order_relaxed);
            p = Pending{};
            return true;
        }
    }
    // silu -> mul(silu, b): complete
    if (p.n == 1 && last->op == gabi::OP_SILU && t->op == gabi::OP_MUL && same_tensor(t->src0, last) && dev_f32(t) &&
        same_shape(t, last) && dev_f32(t->src1) && same_shape(t, t->src1)) {
        const OpTables &tb = op_tables(id, s);
        // one row (decode): hold it for the q4_0 GEMV that follows (norm_fold)
        NormChain c;
        c.kind = 2;
        c.a = (const float *)dptr(last->src0);
        c.b = (const float *)dptr(t->src1);
        c.norm = (float *)dptr(last);
        c.out = (float *)dptr(t);
        c.table = tb.silu;
        c.ncols = t->ne[0];
        auto al = [](const void *q) { return ((uintptr_t)q & 15) == 0; };
        bool fold = silu_fold_enabled() && !exact_mode() && gabi::nrows(t) == 1 && c.ncols % 64 == 0 &&
                    c.ncols <= 16384 && al(c.a) && al(c.b) && al(c.norm) && al(c.out);
        for (const tensor *o : {(const tensor *)last, (const tensor *)t})
            for (const tensor *i : {(const tensor *)last->src0, (const tensor *)t->src1})
                if (dev_overlap(o, i)) fold = false;
        if (x9_chain_ok(c.ncols, gabi::nrows(t)) && t->ne[2] == 1 && t->ne[3] == 1 && al(c.a) && al(c.b) && al(c.norm) &&
            al(c.out)) {
            fold = true;
            c.nrows = gabi::nrows(t);
        }
        if (fold) {
            c.node[c.nn++] = last;
            c.node[c.nn++] = hold(t);
            c.out_node = c.node[1];
            c.on = true;
            g_norm = c;
            p = Pending{};
            return true;
        }
        HIP_FATAL(hipSetDevice(id));
        HIP_FATAL(ghip::op_silu_mul_f32((const float *)dptr(last->src0), (const float *)dptr(t->src1), (float *)dptr(last),
                                        (float *)dptr(t), t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3], tb.silu, s));
        count_node(last);
        count_node(t);
        g_fused[2].fetch_add(1, std::memory_order_relaxed);
        p = Pending{};
        return true;
    }
    // rope -> cpy(rope, strided device view): complete (the K cache store)
    if (p.n == 1 && last->op == gabi::OP_ROPE && t->op == gabi::OP_CPY && same_tensor(t->src0, last) && t->src1 &&
        t->src1->backend == gabi::BACKEND_GPU && t->src1->extra &&
        (t->src1->type == gabi::TYPE_F16 || t->src1->type == gabi::TYPE_F32) && t->src1->ne[3] == 1 &&
        t->src1->ne[0] * t->src1->ne[1] * t->src1->ne[2] == last->ne[0] * last->ne[1] * last->ne[2] &&
        !overlaps(t->src1, last) && !overlaps(t->src1, last->src0)) {
        p = Pending{};
        run_device_op(last, t);
        count_node(t);
        g_fused[3].fetch_add(1, std::memory_order_relaxed);
        return true;
    }
    // f16 mul_mat -> cpy(permute(mul_mat, 0, 2, 1, 3), contiguous f32): complete (KQV_merged_contiguous)
    if (p.n == 1 && last->op == gabi::OP_MUL_MAT && t->op == gabi::OP_CPY && t->src0 && t->src0->op == gabi::OP_PERMUTE &&
        same_tensor(t->src0->src0, last)) {
        const tensor *m = t->src0, *cb = t->src1;
        if (m->ne[0] == last->ne[0] && m->ne[1] == last->ne[2] && m->ne[2] == last->ne[1] && m->ne[3] == 1 &&
            last->ne[3] == 1 && m->nb[0] == 4 && m->nb[1] == last->nb[2] && m->nb[2] == last->nb[1] && dev_f32(cb) &&
            gabi::nbytes(cb) == gabi::nbytes(last) && !overlaps(cb, last) && !overlaps(cb, last->src0) &&
            !overlaps(cb, last->src1)) {
            p = Pending{};
            run_device_op(last, t);
            count_node(t);
            g_fused[4].fetch_add(1, std::memory_order_relaxed);
            return true;
        }
    }
    // pending silu, then a q4_0 mul_mat that neither reads nor overwrites its buffers: run it now
    if (p.n == 1 && last->op == gabi::OP_SILU && t->op == gabi::OP_MUL_MAT && t->src0 &&
        t->src0->type == gabi::TYPE_Q4_0 && t->backend == gabi::BACKEND_GPU && t->src1 &&
        t->src1->backend == gabi::BACKEND_GPU && !overlaps(t->src1, last) && !overlaps(t, last) &&
        !overlaps(t, last->src0)) {
        count_node(t);
        g_fused[5].fetch_add(1, std::memory_order_relaxed);
        mul_mat_node(t->src0, t->src1, t);
        return true;
    }
    return false;
}

// ---- sibling q4_0 GEMVs.  ggml visits a LLaMA layer depth first, so the mul_mats that share an
// input are not adjacent (wk, rope K, cpy K, wv, cpy V, wq, ...; w1, silu, w3).  A q4_0 mul_mat
// with device operands opens a group; the device-only nodes that follow are held
// behind it ("after" nodes, replayed in arrival order once the group has run), and a later q4_0
// mul_mat with the same src1 joins the group when running it ahead of the held nodes is safe: it
// reads none of their outputs and its output overlaps none of their operands.  The group is one
// multi-matrix GEMV launch (ggml_hip_mul_mat_q4_0_multi), bit-identical to separate launches at decode; a
// prefill group on fp6 images is one k_gemm9 launch whose tile plan follows its total tile count (within the
// oracle bound of separate launches; bitwise only with the tile pinned, include/ggml-hip.h).
struct Group {
    int n = 0, na = 0;
    tensor *mm[4] = {};
    tensor *after[16] = {};
    NormChain norm;                // the held norm chain the GEMVs run in their prologue (or off)
};
Group g_grp;
void execute_node(tensor *t);

// last byte + 1 of a device tensor's storage, strides included (views, permutes)
size_t span_bytes(const tensor *t) {
    if (gabi::blck_size(t->type) != 1) return gabi::nbytes(t);
    size_t last = gabi::type_size(t->type);
    for (int i = 0; i < 4; i++) last += (size_t)(t->ne[i] - 1) * t->nb[i];
    return last;
}
bool dev_overlap(const tensor *a, const tensor *b) {
    if (!a || !b || a->backend != gabi::BACKEND_GPU || b->backend != gabi::BACKEND_GPU || !a->extra || !b->extra) return false;
    const char *pa = dptr(a), *pb = dptr(b);
    return pa < pb + span_bytes(b) && pb < pa + span_bytes(a);
}

bool main_device_only_split(int64_t M) {
    int active = 0, only = -1;
    for (int id = 0; id < g_device_count; id++) {
        int64_t lo, hi;
        split_range(M, id, &lo, &hi);
        if (lo < hi) active++, only = id;
    }
    return active == 1 && only == g_main_device;
}

bool group_mm_ok(const tensor *t) {
    if (!fuse_enabled() || t->op != gabi::OP_MUL_MAT || !t->src0 || t->src0->type != gabi::TYPE_Q4_0) return false;
    const tensor *a = t->src0, *b = t->src1;
    if (!b || t->backend != gabi::BACKEND_GPU || !t->extra || b->backend != gabi::BACKEND_GPU || !b->extra || !a->extra)
        return false;
    if (!supported_mul_mat(a, b, t) || !is_contiguous(a) || !is_contiguous(b) || !is_contiguous(t)) return false;
    if (b->ne[1] < 1 || b->ne[2] != 1 || b->ne[3] != 1 || a->ne[2] != 1 || a->ne[3] != 1) return false;
    if (a->backend == gabi::BACKEND_GPU) return true;
    return a->backend == gabi::BACKEND_GPU_SPLIT && main_device_only_split(a->ne[1]);
}

bool group_after_ok(const tensor *t) {
    auto dev = [](const tensor *x) { return x && x->backend == gabi::BACKEND_GPU && x->extra; };
    // a CPY node is a view of its target (src1) that llama.cpp does not hand to assign_buffers:
    // its own backend says nothing, the target's does
    if (t->op != gabi::OP_CPY && !dev(t)) return false;
    switch (t->op) {
        case gabi::OP_ADD:
        case gabi::OP_MUL:
            return dev(t->src0) && dev(t->src1);
        case gabi::OP_SILU:
        case gabi::OP_RMS_NORM:
        case gabi::OP_SOFT_MAX:
            return dev(t->src0);
        case gabi::OP_SCALE:
        case gabi::OP_DIAG_MASK_INF:
        case gabi::OP_ROPE:
            return dev(t->src0) && host_scalar_param(t->src1);
        case gabi::OP_CPY:
            return dev(t->src0) && dev(t->src1);
        case gabi::OP_MUL_MAT:
            return t->src0 && t->src0->type == gabi::TYPE_F16 && dev(t->src0) && dev(t->src1);
        default:
            return false;
    }
}

// may q4_0 mul_mat m run before every held node and beside the current members?
bool norm_feeds(const NormChain &c, const tensor *m);
bool group_join_ok(const tensor *m) {
    const Group &g = g_grp;
    if (g.n >= 4 || !same_tensor(m->src1, g.mm[0]->src1) || m->src0->ne[0] != g.mm[0]->src0->ne[0]) return false;
    if (g.norm.on && !norm_feeds(g.norm, m)) return false;
    for (int i = 0; i < g.n; i++)
        if (dev_overlap(m, g.mm[i]) || dev_overlap(m, g.mm[i]->src1)) return false;
    for (int i = 0; i < g.na; i++) {
        const tensor *A = g.after[i];
        if (dev_overlap(m, A) || dev_overlap(m, A->src0) || dev_overlap(m, A->src1)) return false;
        if (dev_overlap(A, m->src1) || dev_overlap(A, m->src0)) return false;
        if (A->op == gabi::OP_CPY && (dev_overlap(A->src1, m->src1) || dev_overlap(A->src1, m->src0))) return false;
    }
    return true;
}

bool trace_nodes() {
    static const bool on = getenv("GGML_HIP_TRACE_NODES") != nullptr;
    return on;
}

// ---- the independent elementwise nodes a group holds (rope K -> K cache, V -> V cache, rope Q):
// one launch for up to four of them when none reads or writes what another writes
struct ElemRW {
    const tensor *r[2];
    const tensor *w[2];
};
bool dev_t(const tensor *x) { return x && x->backend == gabi::BACKEND_GPU && x->extra; }

bool rope_elem(const tensor *t, ghip::ElemOp &op) {
    const tensor *a = t->src0, *b = t->src1;
    if (t->op != gabi::OP_ROPE || !dev_t(a) || !dev_t(t) || a->type != gabi::TYPE_F32 || t->type != gabi::TYPE_F32 ||
        !host_scalar_param(b))
        return false;
    const int n_past = ((const int32_t *)b->data)[0], n_dims = ((const int32_t *)b->data)[1];
    if (((const int32_t *)b->data)[2] != 0 || !same_shape(a, t) || a->nb[0] != 4 || t->nb[0] != 4 || a->ne[0] % 2 ||
        n_dims % 2 || n_past < 0)
        return false;
    const int64_t np = a->ne[0] / 2;
    const float *cs = rope_table(g_main_device, a->ne[0], n_dims, (int64_t)n_past + a->ne[2], g_dev[g_main_device].stream);
    op = ghip::ElemOp{};
    op.kind = 0;
    op.x = dptr(a);
    op.d = dptr(t);
    op.cs = (const float2 *)(cs + (size_t)n_past * np * 2);
    op.npairs = (int)np;
    op.n = np * a->ne[1] * a->ne[2] * a->ne[3];
    op.ne0 = a->ne[0], op.ne1 = a->ne[1], op.ne2 = a->ne[2];
    op.nbx1 = a->nb[1], op.nbx2 = a->nb[2], op.nbx3 = a->nb[3];
    op.nbd1 = t->nb[1], op.nbd2 = t->nb[2], op.nbd3 = t->nb[3];
    return true;
}
bool cpy_target_ok(const tensor *t) {     // a CPY node F32 -> F32/F16 between device tensors, 3-d
    const tensor *a = t->src0, *b = t->src1;
    return t->op == gabi::OP_CPY && dev_t(a) && dev_t(b) && a->type == gabi::TYPE_F32 &&
           (b->type == gabi::TYPE_F32 || b->type == gabi::TYPE_F16) && a->ne[3] == 1 && b->ne[3] == 1 &&
           a->ne[0] * a->ne[1] * a->ne[2] == b->ne[0] * b->ne[1] * b->ne[2];
}
void set_copy_target(ghip::ElemOp &op, const tensor *b) {
    op.c = dptr(b);
    op.f16 = b->type == gabi::TYPE_F16;
    op.ne10 = b->ne[0], op.ne11 = b->ne[1], op.nb10 = b->nb[0], op.nb11 = b->nb[1], op.nb12 = b->nb[2];
}

// batches a prefix of the held list; returns how many held nodes it ran
int run_elem_prefix(tensor *const *held, int nh) {
    if (!fuse_enabled()) return 0;
    ghip::ElemBatch b{};
    ElemRW rw[ghip::ELEM_MAX];
    int used = 0;
    while (b.nops < ghip::ELEM_MAX && used < nh) {
        tensor *t = held[used];
        ghip::ElemOp op;
        ElemRW e{{nullptr, nullptr}, {nullptr, nullptr}};
        int take = 0;
        if (rope_elem(t, op)) {
            e.r[0] = t->src0;
            e.w[0] = t;
            take = 1;
            if (used + 1 < nh && held[used + 1]->src0 == t && cpy_target_ok(held[used + 1]) &&
                t->ne[3] == 1 && !dev_overlap(held[used + 1]->src1, t) && !dev_overlap(held[used + 1]->src1, t->src0)) {
                set_copy_target(op, held[used + 1]->src1);
                e.w[1] = held[used + 1]->src1;
                take = 2;
            }
        } else if (cpy_target_ok(t)) {
            const tensor *a = t->src0;
            op = ghip::ElemOp{};
            op.kind = 1;
            op.x = dptr(a);
            op.n = a->ne[0] * a->ne[1] * a->ne[2];
            op.ne0 = a->ne[0], op.ne1 = a->ne[1];
            op.nbx1 = a->nb[0], op.nbx2 = a->nb[1], op.nbx3 = a->nb[2];
            set_copy_target(op, t->src1);
            e.r[0] = a;
            e.w[0] = t->src1;
            take = 1;
        } else {
            break;
        }
        // independent of every entry already in the batch (they run concurrently)
        bool ok = true;
        for (int q = 0; q < b.nops && ok; q++)
            for (const tensor *w : rw[q].w)
                for (const tensor *x : {e.r[0], e.r[1], e.w[0], e.w[1]})
                    if (w && x && dev_overlap(w, x)) ok = false;
        for (int q = 0; q < b.nops && ok; q++)
            for (const tensor *w : e.w)
                for (const tensor *x : rw[q].r)
                    if (w && x && dev_overlap(w, x)) ok = false;
        if (!ok) break;
        rw[b.nops] = e;
        b.op[b.nops++] = op;
        used += take;
    }
    if (b.nops < 2) return 0;
    HIP_FATAL(hipSetDevice(g_main_device));
    HIP_FATAL(ghip::op_elem_batch(b, g_dev[g_main_device].stream));
    for (int i = 0; i < used; i++) count_node(held[i]);
    g_fused[7].fetch_add(1, std::memory_order_relaxed);
    return used;
}

void launch_norm_chain(const NormChain &c) {
    const int id = g_main_device;
    HIP_FATAL(hipSetDevice(id));
    if (c.kind == 2)
        HIP_FATAL(ghip::op_silu_mul_f32(c.a, c.b, c.norm, c.out, c.ncols * c.nrows, c.table, g_dev[id].stream));
    else
        HIP_FATAL(ghip::op_add_rms_norm_mul_f32(c.a, c.b, c.sum, c.norm, c.w, c.out, c.ncols, c.nrows, g_dev[id].stream));
    for (int i = 0; i < c.nn; i++) count_node(c.node[i]);
    g_fused[c.kind == 2 ? 2 : 0].fetch_add(1, std::memory_order_relaxed);
}
void flush_norm() {
    const NormChain c = g_norm;
    g_norm = NormChain{};
    if (c.on) launch_norm_chain(c);
}
// may a held norm chain's output feed q4_0 mul_mat m through its GEMV prologue?
bool norm_feeds(const NormChain &c, const tensor *m) {
    if (!c.on || !same_tensor(m->src1, c.out_node) || m->src1->ne[1] != c.nrows || m->src0->ne[0] != c.ncols) return false;
    // m's output must not alias anything the prologue reads or workgroup 0 stores
    const char *y = dptr(m);
    const size_t yb = span_bytes(m), row = (size_t)c.ncols * (size_t)c.nrows * 4;
    for (const void *q : {(const void *)c.a, (const void *)c.b, (const void *)c.w, (const void *)c.sum,
                          (const void *)c.norm, (const void *)c.out})
        if (q && (const char *)q < y + yb && y < (const char *)q + row) return false;
    return true;
}

// prefill (N > IMG_MIN_N) mul_mats of resident weights take k_gemm9 on an fp6 image built once
// (mul_mat_node's rule, here for a group's members)
void ensure_group_images(const Group &g) {
    const int64_t N = g.mm[0]->src1->ne[1];
    if (N <= IMG_MIN_N || exact_mode() || (gemm_version() != 8 && gemm_version() != 10)) return;
    const int id = g_main_device;
    HIP_FATAL(hipSetDevice(id));
    for (int i = 0; i < g.n; i++) wimage_ensure(id, dptr(g.mm[i]->src0), g.mm[i]->src0->ne[0], g.mm[i]->src0->ne[1], g_dev[id].stream);
}

// A held prefill chain and the q4_0 mul_mats that consume it: when every member takes k_gemm9 on an
// fp6 image, the chain's launch writes the x image beside its f32 output and the members run as one
// k_gemm9 launch on it (no k_prep9_x; the image is bitwise gemm9_prep_x's of the chain's output, so y
// is bitwise the unfused path's).  false: not every member qualifies (nothing launched).
bool flush_group_x9(const Group &g) {
    const NormChain &c = g.norm;
    const int id = g_main_device;
    const int64_t K = c.ncols, N = c.nrows;
    if (exact_mode() || gemm_version() != 10 || N * K >= ((int64_t)1 << 31)) return false;
    const void *img[4];
    int64_t M[4], ldy[4];
    float *y[4];
    for (int i = 0; i < g.n; i++) {
        const tensor *a = g.mm[i]->src0;
        int fmt = 0;
        M[i] = ldy[i] = a->ne[1];
        img[i] = wimage_find(id, dptr(a), K, M[i], &fmt);
        if (!img[i] || fmt != 9 || M[i] * (K / QK) * Q4B >= ((int64_t)1 << 31) || M[i] >= (1 << 30)) return false;
        y[i] = (float *)dptr(g.mm[i]);
    }
    hipStream_t s = g_dev[id].stream;
    void *ws = nullptr;
    if (stream_workspace(id, s, workspace_bytes_mm(K, N, 0), &ws) != GGML_HIP_OK) return false;
    void *xws = (char *)ws + ws_g8x_offset(K, N);
    const int64_t Np = ghip::gemm9_np(N);
    HIP_FATAL(hipSetDevice(id));
    if (c.kind == 2)
        HIP_FATAL(ghip::op_silu_mul_f32_x9(c.a, c.b, c.norm, c.out, K, N, c.table, xws, Np, s));
    else
        HIP_FATAL(ghip::op_add_rms_norm_mul_f32_x9(c.a, c.b, c.sum, c.norm, c.w, c.out, K, N, xws, Np, s));
    HIP_FATAL(ghip::gemm9_run_multi(g.n, img, M, K, xws, N, y, ldy, s));
    for (int i = 0; i < c.nn; i++) count_node(c.node[i]);
    for (int i = 0; i < g.n; i++) count_node(g.mm[i]);
    g_fused[c.kind == 2 ? 2 : 0].fetch_add(1, std::memory_order_relaxed);
    g_fused[11].fetch_add(1, std::memory_order_relaxed);
    if (g.n > 1) g_fused[6].fetch_add(1, std::memory_order_relaxed);
    return true;
}

// f32 elements of t at byte offset 4 * (linear element index) from its data (a contiguous, or a
// transposed single-row / single-column, view)
bool linear_f32(const tensor *t) {
    if (t->type != gabi::TYPE_F32) return false;
    int64_t want = 4;
    for (int i = 0; i < 4; i++) {
        if (t->ne[i] > 1 && t->nb[i] != want) return false;
        want *= t->ne[i];
    }
    return true;
}

// The prefix of a decode norm group's held nodes that the GEMV finishes in its epilogue (ghip::GemvEpi):
// each one reads exactly one member's whole output as linear elements (rope mode 0 on one token, with its
// K-cache copy, or a copy such as V into the transposed V cache), at most one per member, and writes
// nothing any member, the norm chain or another of them reads or writes.  Returns how many held nodes
// that is (0: no epilogue).
int epi_prefix(const Group &g, ghip::GemvEpi &ep) {
    if (!fuse_enabled() || !epi_fold_enabled() || g.norm.kind != 1 || g.na == 0) return 0;
    ep = ghip::GemvEpi{};
    struct Range {
        const char *p;
        size_t n;
    };
    std::vector<Range> wr;                 // what the epilogue writes besides the members' outputs
    int owner[4] = {-1, -1, -1, -1};
    auto member_of = [&](const tensor *x) {
        for (int i = 0; i < g.n; i++)
            if (dptr(x) == dptr(g.mm[i]) && x->ne[0] * x->ne[1] * x->ne[2] * x->ne[3] == g.mm[i]->src0->ne[1] &&
                g.mm[i]->src0->ne[1] < ((int64_t)1 << 20) && linear_f32(x))
                return owner[i] < 0 ? i : -1;
        return -1;
    };
    auto add_copy = [&](int i, const tensor *b) {
        // the kernel's index math: extents below 2^20 (udiv20), byte strides in int32
        if (b->ne[0] >= ((int64_t)1 << 20) || b->ne[1] >= ((int64_t)1 << 20) || b->nb[0] > INT32_MAX || b->nb[1] > INT32_MAX ||
            b->nb[2] > INT32_MAX)
            return false;
        ep.c[i] = dptr(b);
        ep.f16[i] = b->type == gabi::TYPE_F16;
        ep.ne10[i] = (int)b->ne[0], ep.ne11[i] = (int)b->ne[1];
        ep.nb10[i] = (int)b->nb[0], ep.nb11[i] = (int)b->nb[1], ep.nb12[i] = (int)b->nb[2];
        wr.push_back({dptr(b), span_bytes(b)});
        return true;
    };
    int used = 0, nops = 0;
    while (used < g.na) {
        const tensor *t = g.after[used];
        ghip::ElemOp op;
        int i = -1, take = 0;
        if (rope_elem(t, op)) {
            i = member_of(t->src0);
            if (i < 0 || t->src0->ne[2] != 1 || !linear_f32(t) || op.ne0 % 2 || op.npairs * 2 != op.ne0) break;
            ep.kind[i] = 1;
            ep.d[i] = (float *)dptr(t);
            ep.cs[i] = op.cs;
            ep.ne0[i] = (int)op.ne0;
            if (dptr(t) != dptr(g.mm[i])) wr.push_back({dptr(t), span_bytes(t)});
            take = 1;
            if (used + 1 < g.na && g.after[used + 1]->src0 == t && cpy_target_ok(g.after[used + 1]) &&
                add_copy(i, g.after[used + 1]->src1))
                take = 2;
        } else if (cpy_target_ok(t)) {
            i = member_of(t->src0);
            if (i < 0) break;
            ep.kind[i] = 2;
            if (!add_copy(i, t->src1)) break;
            take = 1;
        } else {
            break;
        }
        owner[i] = used;
        used += take;
        nops++;
    }
    if (nops == 0) return 0;
    // nothing written overlaps another write, a member's output, or the norm chain's operands
    const size_t row = (size_t)g.norm.ncols * 4;
    std::vector<Range> rd;
    for (int i = 0; i < g.n; i++) rd.push_back({dptr(g.mm[i]), span_bytes(g.mm[i])});
    for (const void *q : {(const void *)g.norm.a, (const void *)g.norm.b, (const void *)g.norm.w,
                          (const void *)g.norm.sum, (const void *)g.norm.norm, (const void *)g.norm.out})
        if (q) rd.push_back({(const char *)q, row});
    auto hit = [](const Range &a, const Range &b) { return a.p < b.p + b.n && b.p < a.p + a.n; };
    for (size_t a = 0; a < wr.size(); a++) {
        for (size_t b = a + 1; b < wr.size(); b++)
            if (hit(wr[a], wr[b])) return 0;
        for (const Range &r : rd)
            if (hit(wr[a], r)) return 0;
    }
    for (int i = 0; i < g.n; i++) {        // rows of members without an op: plain stores
        if (owner[i] >= 0) continue;
        ep.kind[i] = 0;
    }
    return used;
}

// w1 | w3 followed by silu(w1) -> mul(silu, w3) (the LLaMA FFN, held behind the group): the GEMV runs
// the two matrices as interleaved (gate, up) rows and finishes silu -> mul in its epilogue (GemvEpi
// glu).  Returns 2 (the held nodes it takes) and the gate's member index, or 0.
int glu_prefix(const Group &g, ghip::GemvEpi &ep, int *gate) {
    if (!fuse_enabled() || !epi_fold_enabled() || !silu_fold_enabled() || g.norm.kind != 1 || g.n != 2 || g.na < 2)
        return 0;
    const tensor *sl = g.after[0], *ml = g.after[1];
    if (sl->op != gabi::OP_SILU || ml->op != gabi::OP_MUL || !same_tensor(ml->src0, sl) || !dev_f32(sl) || !dev_f32(ml))
        return 0;
    const int64_t M = g.mm[0]->src0->ne[1];
    if (g.mm[1]->src0->ne[1] != M || M >= ((int64_t)1 << 30)) return 0;
    int ga = -1;
    for (int i = 0; i < 2; i++)
        if (dptr(sl->src0) == dptr(g.mm[i])) ga = i;
    if (ga < 0 || dptr(ml->src1) != dptr(g.mm[1 - ga])) return 0;
    for (const tensor *x : {(const tensor *)sl->src0, (const tensor *)ml->src1, sl, ml})
        if (x->type != gabi::TYPE_F32 || x->ne[0] * gabi::nrows(x) != M || !linear_f32(x)) return 0;
    // the two stores write nothing the GEMV, its norm prologue or the other stores touch
    const size_t row = (size_t)g.norm.ncols * 4;
    for (const tensor *o : {(const tensor *)sl, (const tensor *)ml}) {
        for (int i = 0; i < 2; i++)
            if (dev_overlap(o, g.mm[i])) return 0;
        for (const void *q : {(const void *)g.norm.a, (const void *)g.norm.b, (const void *)g.norm.w,
                              (const void *)g.norm.sum, (const void *)g.norm.norm, (const void *)g.norm.out})
            if (q && (const char *)q < dptr(o) + span_bytes(o) && dptr(o) < (const char *)q + row) return 0;
    }
    if (dev_overlap(sl, ml)) return 0;
    ep = ghip::GemvEpi{};
    ep.glu = 1;
    ep.table = op_tables(g_main_device, g_dev[g_main_device].stream).silu;
    ep.d[0] = (float *)dptr(sl);
    ep.d[1] = (float *)dptr(ml);
    *gate = ga;
    return 2;
}

void flush_group() {
    const Group g = g_grp;
    g_grp = Group{};
    if (g.n > 0) ensure_group_images(g);
    if (g.norm.on && g.norm.nrows > 1) {  // a held prefill chain: the x image fold, or its own launch first
        const bool done = flush_group_x9(g);
        if (!done) launch_norm_chain(g.norm);
        if (done) {
            const int k = run_elem_prefix(g.after, g.na);
            for (int i = k; i < g.na; i++) execute_node(g.after[i]);
            return;
        }
    } else if (g.norm.on) {               // the GEMVs run the held norm chain in their prologue
        const void *w[4];
        int64_t m[4], ldy[4];
        float *y[4];
        for (int i = 0; i < g.n; i++) {
            w[i] = dptr(g.mm[i]->src0);
            m[i] = ldy[i] = g.mm[i]->src0->ne[1];
            y[i] = (float *)dptr(g.mm[i]);
        }
        const ghip::GemvNorm nrm{g.norm.a, g.norm.w, g.norm.sum, g.norm.norm, g.norm.out, g.norm.kind, g.norm.table};
        HIP_FATAL(hipSetDevice(g_main_device));
        ghip::GemvEpi ep;
        int gate = 0;
        int ne = glu_prefix(g, ep, &gate);
        if (ne > 0 && gate == 1) {        // the gate first
            std::swap(w[0], w[1]);
            std::swap(m[0], m[1]);
            std::swap(ldy[0], ldy[1]);
            std::swap(y[0], y[1]);
        }
        if (ne == 0) ne = epi_prefix(g, ep);
        hipError_t e = hipErrorInvalidValue;
        if (ne > 0) {                     // the launch shape may refuse the epilogue (nothing launched)
            e = ghip::gemv_q4_0_multi_norm(g.n, w, m, g.norm.ncols, g.norm.b, nrm, y, ldy, g_dev[g_main_device].info,
                                           g_dev[g_main_device].stream, &ep);
            if (e == hipErrorInvalidValue) ne = 0;
            else HIP_FATAL(e);
        }
        if (ne == 0)
            HIP_FATAL(ghip::gemv_q4_0_multi_norm(g.n, w, m, g.norm.ncols, g.norm.b, nrm, y, ldy,
                                                 g_dev[g_main_device].info, g_dev[g_main_device].stream));
        for (int i = 0; i < g.norm.nn; i++) count_node(g.norm.node[i]);
        for (int i = 0; i < g.n; i++) count_node(g.mm[i]);
        for (int i = 0; i < ne; i++) count_node(g.after[i]);
        g_fused[g.norm.kind == 2 ? 2 : 0].fetch_add(1, std::memory_order_relaxed);
        g_fused[g.norm.kind == 2 ? 10 : 9].fetch_add(1, std::memory_order_relaxed);
        if (g.n > 1) g_fused[6].fetch_add(1, std::memory_order_relaxed);
        if (ne > 0) g_fused[ep.glu ? 13 : 12].fetch_add(1, std::memory_order_relaxed);
        const int done = ne + run_elem_prefix(g.after + ne, g.na - ne);
        for (int i = done; i < g.na; i++) execute_node(g.after[i]);
        return;
    }
    if (trace_nodes()) fprintf(stderr, "group flush: %d mul_mats (%s ...), %d held nodes\n", g.n, g.mm[0]->name, g.na);
    if (g.n == 1) {
        count_node(g.mm[0]);
        mul_mat_node(g.mm[0]->src0, g.mm[0]->src1, g.mm[0]);
    } else if (g.n > 1) {
        const void *w[4];
        int64_t m[4];
        float *y[4];
        for (int i = 0; i < g.n; i++) {
            w[i] = dptr(g.mm[i]->src0);
            m[i] = g.mm[i]->src0->ne[1];
            y[i] = (float *)dptr(g.mm[i]);
            count_node(g.mm[i]);
        }
        HIP_FATAL(hipSetDevice(g_main_device));
        const int rc = ggml_hip_mul_mat_q4_0_multi(g.n, w, m, g.mm[0]->src0->ne[0], (const float *)dptr(g.mm[0]->src1),
                                                   g.mm[0]->src1->ne[1], y, g_dev[g_main_device].stream);
        if (rc != GGML_HIP_OK) op_abort(g.mm[0], "sibling q4_0 GEMV group failed");
        g_fused[6].fetch_add(1, std::memory_order_relaxed);
    }
    const int done = run_elem_prefix(g.after, g.na);
    for (int i = done; i < g.na; i++) execute_node(g.after[i]);   // the ordinary path, fusion included
}

// runs (or defers) one taken node; the ith == 0 COMPUTE phase of ggml_hip_compute_forward
void execute_node(tensor *t) {
    const int op = t->op;
    if (op == gabi::OP_RESHAPE || op == gabi::OP_VIEW || op == gabi::OP_PERMUTE || op == gabi::OP_TRANSPOSE) {
        count_node(t);                      // no data touched: a pending chain stays pending
        return;
    }
    if (g_kq) {                             // only the scale of the held KQ may start the chain behind it
        if (g_pend.n == 0 && t->op == gabi::OP_SCALE && same_tensor(t->src0, g_kq) && deferrable(t)) {
            g_pend.node[g_pend.n++] = hold(t);
            return;
        }
        if (g_pend.n == 0) flush_kq();
    }
    if (!g_kq && g_pend.n == 0 && g_grp.n == 0 && !g_norm.on && kq_holdable(t)) {
        g_kq = hold(t);
        return;
    }
    // a held norm chain: a GEMV that consumes it opens a group that runs it in its prologue
    auto open_norm_group = [&]() {
        if (!g_norm.on || g_grp.n != 0 || g_pend.n != 0 || !group_mm_ok(t) || !norm_feeds(g_norm, t)) return false;
        g_grp.mm[0] = hold(t);
        g_grp.n = 1;
        g_grp.norm = g_norm;
        g_norm = NormChain{};
        return true;
    };
    if (g_norm.on) {
        if (open_norm_group()) return;
        flush_norm();                         // anything else: the chain runs as its own launch
    }
    if (g_grp.n > 0) {
        if (group_mm_ok(t) && group_join_ok(t)) {
            g_grp.mm[g_grp.n++] = hold(t);
            return;
        }
        if (trace_nodes())
            fprintf(stderr, "group: %s not joined (mm_ok %d, join_ok %d, after_ok %d)\n", t->name, (int)group_mm_ok(t),
                    group_mm_ok(t) ? (int)group_join_ok(t) : -1, (int)group_after_ok(t));
        if (!(op == gabi::OP_MUL_MAT && t->src0 && t->src0->type != gabi::TYPE_F16) && group_after_ok(t) &&
            g_grp.na < 16) {
            g_grp.after[g_grp.na++] = hold(t);
            return;
        }
        flush_group();                        // its held nodes may complete a norm chain t consumes
        if (open_norm_group()) return;
        if (g_norm.on) flush_norm();
    }
    if (g_pend.n == 0 && group_mm_ok(t)) {
        g_grp.mm[0] = hold(t);
        g_grp.n = 1;
        return;
    }
    if (g_pend.n > 0) {
        if (try_fuse(t)) return;
        flush_pending();
        if (group_mm_ok(t)) {
            g_grp.mm[0] = hold(t);
            g_grp.n = 1;
            return;
        }
    }
    if (deferrable(t)) {
        g_pend.node[g_pend.n++] = hold(t);
        return;
    }
    if (t->op == gabi::OP_MUL_MAT && t->src0 && t->src0->type != gabi::TYPE_F16) {
        count_node(t);
        ggml_hip_mul_mat((const ggml_tensor *)t->src0, (const ggml_tensor *)t->src1, (ggml_tensor *)t);
    } else {
        run_device_op(t);
    }
}

}  // namespace ghh

namespace ghh {

// every backend entry point that can touch device memory outside the node sequence
// launch recording on the hook path: opt-in (GGML_HIP_GRAPH=1 or ggml_hip_debug_set_graph(1)).  It cuts
// the host walk of a LLaMA-7B decode eval from 1.36 to 0.59 ms, but the eval is device bound (~330
// kernels, ~2.3 us per boundary) and HIP's graph replay leaves a ~100 us gap every 16 nodes: equal or
// 2-3 % slower end to end, so eager launches stay the default.
std::atomic<int> &graph_flag() {
    static std::atomic<int> f([] {
        const char *e = getenv("GGML_HIP_GRAPH");
        return e ? atoi(e) : 0;
    }());
    return f;
}
bool graph_enabled() { return graph_flag().load(std::memory_order_relaxed) != 0; }
int graph_apply_mode() {           // 1: HIP graphs, 2: launcher thread, 3: own AQL queue (launch.h); returns the mode
    static int applied = -1;
    const int m = graph_flag().load(std::memory_order_relaxed);
    if (m != applied && m != 0) ghip::rec_set_mode(m);
    applied = m;
    return m == 2 || m == 3 ? m : (m != 0 ? 1 : 0);
}

bool hook_holding() { return g_grp.n != 0 || g_pend.n != 0 || g_norm.on || g_kq; }
bool hook_seen(const tensor *t) { return g_snaps.memo.count(t) != 0; }

void flush_deferred() {
    if (g_grp.n > 0) flush_group();
    if (g_norm.on) flush_norm();
    if (g_pend.n > 0) flush_pending();
    flush_kq();
    ghip::rec_flush_at("entry point");        // and submit the recorded launches (launch.h)
}

}  // namespace ghh

extern "C" {

// not in the public header: launch-recorder counters (launch.h) — out[0] submitted runs, [1] kernels in
// them, [2] graph nodes updated in place, [3] graphs instantiated, [4] host ns spent submitting;
// clear != 0 also destroys the cache
int ggml_hip_debug_graph_stats(long long *out, int clear) {
    flush_deferred();
    ghip::rec_stats(&out[0], &out[1], &out[2], &out[3], &out[4]);
    if (clear) ghip::rec_clear_cache();
    return GGML_HIP_OK;
}

// not in the public header: host cost of eager launches: out[0] launches, out[1] ns inside hipLaunchKernel;
// enable 1 starts counting (and resets), 0 stops, -1 only reads
int ggml_hip_debug_launch_stats(long long *out, int enable) {
    flush_deferred();
    ghip::launch_prof_read(&out[0], &out[1], enable == 1);
    if (enable >= 0) ghip::g_launch_prof = enable != 0;
    return GGML_HIP_OK;
}

// not in the public header: AQL launch mode counters: out[0] dispatches through the own queue, out[1] launches that
// fell back to hipLaunchKernel, out[2] queue drains (host waits), out[3] host waits for the HIP stream
int ggml_hip_debug_aql_stats(long long *out) {
    ghip::aql_counts(out);
    return GGML_HIP_OK;
}

// not in the public header: every launch_k on `stream` through the launch recorder in `mode` (3: the own AQL queue,
// ggml-hip-aql.cpp), 0 = back to eager HIP launches (drains first); for the tensor-free callers (bench.py's decode)
int ggml_hip_debug_set_stream_launch_mode(void *stream, int mode) {
    flush_deferred();
    if (mode != 0 && mode != 3) return fail(GGML_HIP_ERR_INVALID, "mode must be 0 or 3");
    hipStream_t s = resolve_stream(stream);
    if (mode == 0) {
        ghip::rec_enable(s, false);
        ghip::rec_set_mode(1);
        return GGML_HIP_OK;
    }
    ghip::rec_set_mode(3);
    ghip::rec_enable(s, true);
    return GGML_HIP_OK;
}

// not in the public header: a busy wait of ns nanoseconds after every eager launch (0 = none): the end-to-end
// token time's sensitivity to the host's per-launch cost (tools/e2e_llama.py modes "-padN")
int ggml_hip_debug_set_launch_pad(int ns) {
    flush_deferred();
    ghip::g_launch_pad_ns.store(ns < 0 ? 0 : ns, std::memory_order_relaxed);
    return GGML_HIP_OK;
}

// not in the public header: the decode norm chain folded into the GEMV prologue on (1) / off (0)
int ggml_hip_debug_set_norm_fold(int on) {
    flush_deferred();
    g_norm_fold.store(on < 0 || on > 2 ? 1 : on);
    return GGML_HIP_OK;
}

// not in the public header: the decode q|k|v GEMV epilogue (held rope / copy nodes) on (1) / off (0)
int ggml_hip_debug_set_epi_fold(int on) {
    flush_deferred();
    g_epi_fold.store(on ? 1 : 0);
    return GGML_HIP_OK;
}

// not in the public header: the decode KQ computed by the soft_max -> KQV launch on (1) / off (0)
int ggml_hip_debug_set_kq_fold(int on) {
    flush_deferred();
    g_kq_fold.store(on ? 1 : 0);
    return GGML_HIP_OK;
}

// not in the public header: the prefill x image fold (a held norm / silu chain writes the k_gemm9 x image
// of its output for the q4_0 mul_mats that consume it) on (1) / off (0)
int ggml_hip_debug_set_x9_fold(int on) {
    flush_deferred();
    g_x9_fold.store(on ? 1 : 0);
    return GGML_HIP_OK;
}

// not in the public header: launch recording for the hook path: 0 off, 1 HIP graphs, 2 launcher thread, 3 own AQL
// queue (ggml-hip-aql.cpp)
int ggml_hip_debug_set_graph(int on) {
    flush_deferred();
    graph_flag().store(on);
    return GGML_HIP_OK;
}

}  // extern "C"

extern "C" {

// not in the public header: launch fusion of full-offload chains on (1) / off (0) (tests run both)
int ggml_hip_debug_set_fuse(int on) {
    flush_deferred();
    g_fuse.store(on ? 1 : 0, std::memory_order_relaxed);
    return GGML_HIP_OK;
}

}  // extern "C"
