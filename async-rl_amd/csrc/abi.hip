// C ABI of libasyncrl_hip.so (declared in include/asyncrl_hip.h).
// Argument validation lives here; kernels assume validated shapes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <string>

#include "../../include/asyncrl_hip.h"
#include "arl_internal.hpp"

struct arl_net {
  arl::Net net;
  bool bound = false;
  struct Pool {
    uintptr_t base = 0;
    int64_t bytes = 0;
  };
  Pool pools[3][8];   // registered input pools per kind (arl_net_set_pool)
};

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int hip_status(hipError_t e, const char* what) {
  if (e == hipSuccess) return ARL_OK;
  return fail(ARL_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}
bool aligned(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }
hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }
}  // namespace

extern "C" {

int arl_abi_version(void) { return ARL_ABI_VERSION; }
const char* arl_last_error(void) { return g_err.c_str(); }

int arl_current_screen(const uint8_t* cur, const uint8_t* prev, uint8_t* out, int64_t n, int mode, void* s) {
  if (n < 0 || (n > 0 && (!cur || !prev || !out))) return fail(ARL_EINVAL, "current_screen: null pointer / n < 0");
  if (!aligned(cur, 16) || !aligned(prev, 16) || !aligned(out, 4))
    return fail(ARL_EINVAL, "current_screen: frames must be 16-byte aligned, out 4-byte aligned");
  if (mode < 0 || mode > (ARL_RESIZE_SIMD | ARL_RESIZE_CROP)) return fail(ARL_EINVAL, "bad resize_mode");
  if (n > 65535) return fail(ARL_EINVAL, "current_screen: n > 65535 per call");
  return hip_status(arl::launch_current_screen(cur, prev, out, n, mode, S(s)), "current_screen");
}

int arl_max_luminance(const uint8_t* cur, const uint8_t* prev, uint8_t* gray, int64_t npix, void* s) {
  if (npix < 0 || (npix > 0 && (!cur || !prev || !gray))) return fail(ARL_EINVAL, "max_luminance: null / npix < 0");
  if (npix > ((int64_t)1 << 31) * 255) return fail(ARL_EINVAL, "max_luminance: npix too large");
  return hip_status(arl::launch_max_luminance(cur, prev, gray, npix, S(s)), "max_luminance");
}

int arl_phi_stack(const uint8_t* pairs, const uint8_t* prev_stack, const uint8_t* reset, uint8_t* out_stack,
                  int64_t n, int mode, void* s) {
  if (n < 0 || (n > 0 && (!pairs || !prev_stack || !out_stack)))
    return fail(ARL_EINVAL, "phi_stack: null pointer / n < 0");
  if (!aligned(pairs, 16) || !aligned(prev_stack, 16) || !aligned(out_stack, 16))
    return fail(ARL_EINVAL, "phi_stack: buffers must be 16-byte aligned");
  if (prev_stack == out_stack && n > 0) return fail(ARL_EINVAL, "phi_stack: prev_stack and out_stack alias");
  if (mode < 0 || mode > (ARL_RESIZE_SIMD | ARL_RESIZE_CROP)) return fail(ARL_EINVAL, "bad resize_mode");
  if (n > 65535) return fail(ARL_EINVAL, "phi_stack: n > 65535 per call");
  return hip_status(arl::launch_phi_stack(pairs, prev_stack, reset, out_stack, n, mode, S(s)), "phi_stack");
}

int arl_dqn_phi(const uint8_t* in, float* out, int64_t n, void* s) {
  if (n < 0 || (n > 0 && (!in || !out))) return fail(ARL_EINVAL, "dqn_phi: null pointer / n < 0");
  if (!aligned(in, 4) || !aligned(out, 16)) return fail(ARL_EINVAL, "dqn_phi: in 4-byte, out 16-byte aligned");
  return hip_status(arl::launch_dqn_phi(in, out, n * 4 * arl::PLANE, S(s)), "dqn_phi");
}

static int check_rgb_dims(int H, int W) {
  if (H < 2 || W < 16 || W % 16 != 0 || W > arl::RGB_MAX_W || H > 65535)
    return fail(ARL_EINVAL, "rgb: need H >= 2, W % 16 == 0, 16 <= W <= 2048");
  return ARL_OK;
}

int arl_rgb_phi(const uint8_t* imgs, int64_t n, int H, int W, float* out, int mode, void* s) {
  if (n < 0 || (n > 0 && (!imgs || !out))) return fail(ARL_EINVAL, "rgb_phi: null pointer / n < 0");
  if (int rc = check_rgb_dims(H, W)) return rc;
  if (n > 65535) return fail(ARL_EINVAL, "rgb_phi: n > 65535");
  if (!aligned(imgs, 16) || !aligned(out, 16)) return fail(ARL_EINVAL, "rgb_phi: 16-byte alignment");
  if (mode < 0 || mode > ARL_RESIZE_SIMD) return fail(ARL_EINVAL, "rgb_phi: resize_mode must be 0 or 1");
  return hip_status(arl::launch_rgb_phi(imgs, n, H, W, out, mode, S(s)), "rgb_phi");
}

int arl_net_create(arl_net** out, int arch, int n_actions, int n_envs, int t_max, int env_offset, uint64_t seed) {
  if (!out) return fail(ARL_EINVAL, "net_create: out is null");
  arl_net* h = new arl_net();
  std::string err;
  if (!arl::net_init(h->net, arch, n_actions, n_envs, t_max, env_offset, seed, err)) {
    delete h;
    return fail(ARL_EINVAL, "net_create: " + err);
  }
  *out = h;
  return ARL_OK;
}

void arl_net_destroy(arl_net* h) {
  if (h && h->net.stamps) {
    for (hipEvent_t e : h->net.stamps->ev) (void)hipEventDestroy(e);
    delete h->net.stamps;
  }
  delete h;
}

int64_t arl_net_param_floats(const arl_net* h) { return h ? h->net.param_floats : -1; }
int arl_net_param_count(const arl_net* h) { return h ? (int)h->net.params.size() : -1; }

int arl_net_param_info(const arl_net* h, int idx, int64_t* offset, int64_t* numel, char* name, int cap) {
  if (!h || idx < 0 || idx >= (int)h->net.params.size()) return fail(ARL_EINVAL, "param_info: bad index");
  const arl::ParamInfo& p = h->net.params[idx];
  if (offset) *offset = p.offset;
  if (numel) *numel = p.numel;
  if (name && cap > 0) {
    strncpy(name, p.name.c_str(), (size_t)cap - 1);
    name[cap - 1] = 0;
  }
  return ARL_OK;
}

int64_t arl_net_workspace_bytes(const arl_net* h) { return h ? h->net.ws_bytes : -1; }

int arl_net_buffer(const arl_net* h, const char* name, int64_t* offset, int64_t* bytes) {
  if (!h || !name) return fail(ARL_EINVAL, "net_buffer: null");
  for (const auto& b : h->net.bufs)
    if (strcmp(b.name, name) == 0) {
      if (offset) *offset = b.off;
      if (bytes) *bytes = b.bytes;
      return ARL_OK;
    }
  return fail(ARL_EINVAL, std::string("net_buffer: unknown buffer ") + name);
}

int arl_net_bind(arl_net* h, float* params, float* grads, float* ms, void* ws) {
  if (!h || !params || !grads || !ms || !ws) return fail(ARL_EINVAL, "net_bind: null pointer");
  if (!aligned(params, 16) || !aligned(grads, 16) || !aligned(ms, 16) || !aligned(ws, 256))
    return fail(ARL_EINVAL, "net_bind: params/grads/ms 16-byte aligned, workspace 256-byte aligned");
  h->net.p = params;
  h->net.g = grads;
  h->net.ms = ms;
  h->net.ws = reinterpret_cast<char*>(ws);
  ++h->net.param_gen;   // new parameter memory: derived state (the FC planes) is stale
  h->bound = true;
  return ARL_OK;
}

int arl_net_params_changed(arl_net* h) {
  if (!h) return fail(ARL_EINVAL, "null net");
  ++h->net.param_gen;
  return ARL_OK;
}

int arl_net_param_generation(const arl_net* h, uint64_t* param_gen, uint64_t* planes_gen) {
  if (!h) return fail(ARL_EINVAL, "null net");
  if (param_gen) *param_gen = h->net.param_gen;
  if (planes_gen) *planes_gen = h->net.planes_gen;
  return ARL_OK;
}

#define NEED_BOUND(h)                                                         \
  do {                                                                        \
    if (!(h)) return fail(ARL_EINVAL, "null net");                            \
    if (!(h)->bound) return fail(ARL_ESTATE, "net not bound (arl_net_bind)"); \
  } while (0)

int arl_net_prepare(arl_net* h, void* s) {
  NEED_BOUND(h);
  return hip_status(arl::ensure_fc_planes(h->net, S(s)), "net_prepare");
}

int arl_net_reset(arl_net* h, void* s) {
  NEED_BOUND(h);
  arl::Net& n = h->net;
  hipError_t e = hipMemsetAsync(n.ws + n.w_ctl, 0, arl::CTL_SIZE * 8, S(s));
  if (e == hipSuccess) e = hipMemsetAsync(n.ws + n.w_nvalid, 0, (size_t)n.R * n.N, S(s));
  if (e == hipSuccess) e = hipMemsetAsync(n.ws + n.w_reset, 1, (size_t)(n.T + 1) * n.N, S(s));
  if (e == hipSuccess) e = hipMemsetAsync(n.ws + n.w_tick, 0, (size_t)arl::fc_fwd_tiles(n.N) * 4, S(s));
  if (e == hipSuccess) e = hipMemsetAsync(n.ws + n.w_norm, 0, (size_t)arl::NORM_SCRATCH * 8, S(s));
  if (e == hipSuccess && n.w_fcb_tick)
    e = hipMemsetAsync(n.ws + n.w_fcb_tick, 0, (size_t)arl::fc_bwd_tickets() * 4, S(s));
  n.returns_done = false;
  if (e == hipSuccess && n.arch == arl::ARCH_LSTM) {
    e = hipMemsetAsync(n.ws + n.w_hbuf, 0, (size_t)(n.T + 2) * n.N * arl::HID * 4, S(s));
    if (e == hipSuccess) e = hipMemsetAsync(n.ws + n.w_cbuf, 0, (size_t)(n.T + 2) * n.N * arl::HID * 4, S(s));
    if (e == hipSuccess) e = hipMemsetAsync(n.ws + n.w_eval_reset, 1, (size_t)n.N, S(s));
    if (e == hipSuccess) e = hipMemsetAsync(n.ws + n.w_zero, 0, arl::ZERO_ROW_FLOATS * 4, S(s));
  }
  return hip_status(e, "net_reset");
}

int arl_net_set_pool(arl_net* h, int kind, const void* pool, int64_t bytes) {
  if (!h) return fail(ARL_EINVAL, "null net");
  if (kind < ARL_POOL_FRAMES || kind > ARL_POOL_DONES) return fail(ARL_EINVAL, "set_pool: unknown pool kind");
  if (!pool || bytes < 0) return fail(ARL_EINVAL, "set_pool: null pool / bytes < 0");
  const uintptr_t b = reinterpret_cast<uintptr_t>(pool);
  arl_net::Pool* tab = h->pools[kind];
  int slot = -1;
  for (int i = 0; i < 8; ++i)
    if (tab[i].base == b) slot = i;
  if (slot < 0) {   // a free slot, else replace the oldest registration (slots shift down)
    for (int i = 0; i < 8 && slot < 0; ++i)
      if (tab[i].bytes == 0) slot = i;
    if (slot < 0) {
      for (int i = 0; i < 7; ++i) tab[i] = tab[i + 1];
      slot = 7;
    }
  }
  tab[slot].base = bytes > 0 ? b : 0;
  tab[slot].bytes = bytes;
  // a registration overlapping the new one belongs to memory that was freed and reused: drop it
  for (int i = 0; i < 8 && bytes > 0; ++i)
    if (i != slot && tab[i].bytes > 0 && tab[i].base < b + (uintptr_t)bytes && b < tab[i].base + (uintptr_t)tab[i].bytes)
      tab[i] = arl_net::Pool{};
  return ARL_OK;
}

// a non-null pool must lie inside a registered pool of its kind with pool_len * rows * unit bytes
// before that pool's end (0 = ok)
static int check_pool(const arl_net* h, int kind, const void* pool, int64_t pool_len, int64_t unit, const char* what) {
  if (!pool) return 0;
  const uintptr_t p = reinterpret_cast<uintptr_t>(pool);
  // the registration with the greatest base <= p whose range holds p: a stale, larger registration of a
  // freed pool that also spans p never lends its room to a newer pool allocated inside it
  const arl_net::Pool* best = nullptr;
  for (const arl_net::Pool& r : h->pools[kind]) {
    if (r.bytes <= 0 || p < r.base || p >= r.base + (uintptr_t)r.bytes) continue;
    if (!best || r.base > best->base) best = &r;
  }
  if (!best) return fail(ARL_EINVAL, std::string("observe: the ") + what + " pool is not registered (arl_net_set_pool)");
  const int64_t room = (int64_t)(best->base + (uintptr_t)best->bytes - p);
  if (unit > 0 && pool_len > room / unit)
    return fail(ARL_EINVAL, std::string("observe: pool_len ") + std::to_string(pool_len) + " exceeds the " + what +
                                " pool (" + std::to_string(room / unit) + " entries registered)");
  return 0;
}

// validates an observation and fills its ring arguments (0 = ok)
static int ring_args(arl_net* h, int t, const uint8_t* pool, const float* reward_pool, const uint8_t* done_pool,
                     int64_t pool_len, int force_reset, int mode, int H, int W, int e0, int ne, arl::RingArgs& a) {
  arl::Net& n = h->net;
  if (t < 0 || t > n.T) return fail(ARL_EINVAL, "observe: t out of [0, t_max]");
  if ((!pool && n.layout != arl::FRAMES_STACK && n.layout != arl::FRAMES_STATES) || pool_len < 1)
    return fail(ARL_EINVAL, "observe: need the frame pool and pool_len >= 1");
  if (!aligned(pool, 16)) return fail(ARL_EINVAL, "observe: the frame pool must be 16-byte aligned");
  if (n.N > 65535) return fail(ARL_EINVAL, "observe: n_envs > 65535");
  const int64_t frame_unit = n.layout == arl::FRAMES_RGB ? (int64_t)H * W * 3
                             : n.layout == arl::FRAMES_STACK ? 4 * arl::PLANE
                             : n.layout == arl::FRAMES_STATES ? 16 * arl::PLANE
                                                             : arl::PAIR;
  if (int rc = check_pool(h, ARL_POOL_FRAMES, pool, pool_len, frame_unit * n.N, "frame")) return rc;
  if (int rc = check_pool(h, ARL_POOL_REWARDS, reward_pool, pool_len, 4 * (int64_t)n.N, "reward")) return rc;
  if (int rc = check_pool(h, ARL_POOL_DONES, done_pool, pool_len, (int64_t)n.N, "done")) return rc;
  a.pair_pool = pool;
  a.reward_pool = reward_pool;
  a.done_pool = done_pool;
  a.pool_len = pool_len;
  a.frames = n.at<uint8_t>(n.w_frames);
  a.nvalid = n.at<uint8_t>(n.w_nvalid);
  a.reset_flags = n.at<uint8_t>(n.w_reset);
  a.rewards = n.at<float>(n.w_rewards);
  a.dones = n.at<uint8_t>(n.w_dones);
  a.ctl = n.at<int64_t>(n.w_ctl);
  a.n = n.N;
  a.R = n.R;
  a.t = t;
  a.mode = mode;
  a.force_reset = force_reset ? 1 : 0;
  a.H = H;
  a.W = W;
  a.e0 = e0;
  a.ne = ne;
  a.esize = n.layout == arl::FRAMES_STATES ? 4 : 1;
  return 0;
}

static int observe_common(arl_net* h, int t, const uint8_t* pool, const float* reward_pool,
                          const uint8_t* done_pool, int64_t pool_len, int force_reset, int mode, int H, int W,
                          void* s, int e0 = 0, int ne = -1) {
  arl::RingArgs a;
  if (int rc = ring_args(h, t, pool, reward_pool, done_pool, pool_len, force_reset, mode, H, W, e0, ne, a)) return rc;
  const arl::Net& n = h->net;
  hipError_t e = n.layout == arl::FRAMES_RGB ? arl::launch_rgb_ring(a, S(s))
                 : (n.layout == arl::FRAMES_STACK || n.layout == arl::FRAMES_STATES) ? arl::launch_stack_ring(a, S(s))
                                                                                    : arl::launch_phi_ring(a, S(s));
  if (e == hipSuccess) e = arl::stamp(n, arl::STAGE_PHI, S(s));
  return hip_status(e, "observe");
}

int arl_observe(arl_net* h, int t, const uint8_t* pair_pool, const float* reward_pool, const uint8_t* done_pool,
                int64_t pool_len, int force_reset, int mode, void* s) {
  NEED_BOUND(h);
  if (h->net.rgb) return fail(ARL_ESTATE, "observe: RGB net, use arl_observe_rgb");
  if (h->net.stack) return fail(ARL_ESTATE, "observe: ARL_ARCH_STACK net, use arl_observe_stack");
  if (h->net.states) return fail(ARL_ESTATE, "observe: ARL_ARCH_STATES net, use arl_observe_states");
  if (mode < 0 || mode > (ARL_RESIZE_SIMD | ARL_RESIZE_CROP)) return fail(ARL_EINVAL, "bad resize_mode");
  return observe_common(h, t, pair_pool, reward_pool, done_pool, pool_len, force_reset, mode, 0, 0, s);
}

int arl_observe_rgb(arl_net* h, int t, const uint8_t* img_pool, int H, int W, const float* reward_pool,
                    const uint8_t* done_pool, int64_t pool_len, int force_reset, int mode, void* s) {
  NEED_BOUND(h);
  if (!h->net.rgb) return fail(ARL_ESTATE, "observe_rgb: net was not created with ARL_ARCH_RGB");
  if (mode < 0 || mode > ARL_RESIZE_SIMD) return fail(ARL_EINVAL, "observe_rgb: resize_mode must be 0 or 1");
  if (int rc = check_rgb_dims(H, W)) return rc;
  return observe_common(h, t, img_pool, reward_pool, done_pool, pool_len, force_reset, mode, H, W, s);
}

int arl_observe_stack(arl_net* h, int t, const uint8_t* stack_pool, const float* reward_pool,
                      const uint8_t* done_pool, int64_t pool_len, int force_reset, void* s) {
  NEED_BOUND(h);
  if (!h->net.stack) return fail(ARL_ESTATE, "observe_stack: net was not created with ARL_ARCH_STACK");
  if (!stack_pool && t < 1) return fail(ARL_EINVAL, "observe_stack: a frameless observation needs t >= 1");
  return observe_common(h, t, stack_pool, reward_pool, done_pool, pool_len, force_reset, 0, 0, 0, s);
}

int arl_observe_states(arl_net* h, int t, const float* state_pool, const float* reward_pool,
                       const uint8_t* done_pool, int64_t pool_len, int force_reset, void* s) {
  NEED_BOUND(h);
  if (!h->net.states) return fail(ARL_ESTATE, "observe_states: net was not created with ARL_ARCH_STATES");
  if (!state_pool && t < 1) return fail(ARL_EINVAL, "observe_states: a stateless observation needs t >= 1");
  return observe_common(h, t, reinterpret_cast<const uint8_t*>(state_pool), reward_pool, done_pool, pool_len,
                        force_reset, 0, 0, 0, s);
}

int arl_truncate_window(arl_net* h, int t_len, void* s) {
  NEED_BOUND(h);
  arl::Net& n = h->net;
  if (t_len < 1 || t_len > n.T) return fail(ARL_EINVAL, "truncate_window: t_len out of [1, t_max]");
  n.returns_done = false;   // a truncated window's learn runs its own returns
  if (t_len == n.T) return ARL_OK;
  const size_t rows = (size_t)(n.T - t_len) * n.N;
  hipError_t e = hipMemsetAsync(n.ws + n.w_dones + (size_t)t_len * n.N, 2, rows, S(s));
  if (e == hipSuccess) e = hipMemsetAsync(n.ws + n.w_rewards + (size_t)t_len * n.N * 4, 0, rows * 4, S(s));
  return hip_status(e, "truncate_window");
}

int arl_net_set_norm_fold(arl_net* h, int on) {
  if (!h) return fail(ARL_EINVAL, "null net");
  h->net.norm_fold = on != 0;
  h->net.norm_ready = false;
  return ARL_OK;
}

int arl_net_set_returns_fusion(arl_net* h, int on, double gamma, double beta, double v_loss_coef, int clip_reward) {
  if (!h) return fail(ARL_EINVAL, "null net");
  arl::Net& n = h->net;
  n.fuse_returns = on != 0 && n.arch == arl::ARCH_FF;
  if (on) {   // (turning it off keeps returns_done: the window's learn still skips what the act ran)
    n.returns_done = false;
    n.ret = arl::Net::ReturnsCfg{gamma, (float)beta, (float)v_loss_coef, clip_reward};
  }
  return ARL_OK;
}

int arl_net_set_loss(arl_net* h, double pi_loss_coef, int keep_loss_scale_same) {
  if (!h) return fail(ARL_EINVAL, "null net");
  h->net.pi_coef = (float)pi_loss_coef;
  h->net.keep_scale = keep_loss_scale_same ? 1 : 0;
  return ARL_OK;
}

int arl_act(arl_net* h, int t, void* s) {
  NEED_BOUND(h);
  if (t < 0 || t > h->net.T) return fail(ARL_EINVAL, "act: t out of [0, t_max]");
  return hip_status(arl::net_act(h->net, t, 1, S(s)), "act");
}

int arl_act_mode(arl_net* h, int t, int mode, void* s) {
  NEED_BOUND(h);
  if (t < 0 || t > h->net.T) return fail(ARL_EINVAL, "act: t out of [0, t_max]");
  if (mode < 0 || mode > 2) return fail(ARL_EINVAL, "act: mode must be 0 (none), 1 (sample) or 2 (greedy)");
  return hip_status(arl::net_act(h->net, t, mode, S(s)), "act");
}

static int check_env_range(const arl::Net& n, int e0, int ne) {
  if (ne < 1 || e0 < 0 || e0 > n.N - ne) return fail(ARL_EINVAL, "env range [e0, e0 + ne) outside [0, n_envs)");
  if (e0 % ARL_ENV_GROUP_ALIGN) return fail(ARL_EINVAL, "env range: e0 must be a multiple of ARL_ENV_GROUP_ALIGN");
  if ((n.arch == arl::ARCH_FF_NATURE || n.states) && (e0 != 0 || ne != n.N))
    return fail(ARL_EINVAL, "env range: Nature-head and ARL_ARCH_STATES nets run all envs in one launch");
  return 0;
}

int arl_observe_envs(arl_net* h, int t, int e0, int ne, const uint8_t* pool, int H, int W, const float* reward_pool,
                     const uint8_t* done_pool, int64_t pool_len, int force_reset, int mode, void* s) {
  NEED_BOUND(h);
  if (int rc = check_env_range(h->net, e0, ne)) return rc;
  if (h->net.rgb) {
    if (mode < 0 || mode > ARL_RESIZE_SIMD) return fail(ARL_EINVAL, "observe_rgb: resize_mode must be 0 or 1");
    if (int rc = check_rgb_dims(H, W)) return rc;
  } else if (h->net.stack || h->net.states) {
    H = W = mode = 0;
  } else {
    if (mode < 0 || mode > (ARL_RESIZE_SIMD | ARL_RESIZE_CROP)) return fail(ARL_EINVAL, "bad resize_mode");
    H = W = 0;
  }
  return observe_common(h, t, pool, reward_pool, done_pool, pool_len, force_reset, mode, H, W, s, e0, ne);
}

int arl_act_envs(arl_net* h, int t, int e0, int ne, int mode, void* s) {
  NEED_BOUND(h);
  if (t < 0 || t > h->net.T) return fail(ARL_EINVAL, "act: t out of [0, t_max]");
  const int part = mode & ~3;
  if (mode < 0 || (mode & 3) > 2 || (part != 0 && part != ARL_ACT_CONV_ONLY && part != ARL_ACT_AFTER_CONV))
    return fail(ARL_EINVAL, "act: mode must be 0 / 1 / 2, optionally | ARL_ACT_CONV_ONLY or ARL_ACT_AFTER_CONV");
  if (int rc = check_env_range(h->net, e0, ne)) return rc;
  if (part != 0 && h->net.arch == arl::ARCH_FF_NATURE) return fail(ARL_EINVAL, "act: Nature head has no conv split");
  if (ne != h->net.N && !h->net.planes_current() && h->net.arch != arl::ARCH_FF_NATURE)
    return fail(ARL_ESTATE, "act: the params changed since the FC weight planes were built; call arl_net_prepare on "
                            "the stream the env-range chains fork from before issuing them");
  return hip_status(arl::net_act(h->net, t, mode, S(s), e0, ne), "act");
}

int arl_run_stage(arl_net* h, int stage, int t, void* s) {
  NEED_BOUND(h);
  if (stage < ARL_STAGE_CONV_FWD || (stage > ARL_STAGE_LSTM_WGRAD && stage != ARL_STAGE_RMSPROP))
    return fail(ARL_EINVAL, "run_stage: unknown stage");
  if (stage >= ARL_STAGE_RETURNS && h->net.arch == arl::ARCH_FF_NATURE)
    return fail(ARL_EINVAL, "run_stage: returns / conv reduce / grad sqnorm stages are NIPS-head only");
  if (stage >= ARL_STAGE_LSTM_GATES && stage <= ARL_STAGE_LSTM_WGRAD && h->net.arch != arl::ARCH_LSTM)
    return fail(ARL_EINVAL, "run_stage: the LSTM stages need an LSTM net");
  if (t < 0 || t > h->net.T) return fail(ARL_EINVAL, "run_stage: t out of [0, t_max]");
  return hip_status(arl::net_stage(h->net, stage, t, S(s)), "run_stage");
}

int arl_stamps_begin(arl_net* h, int cap) {
  NEED_BOUND(h);
  if (cap < 1 || cap > (1 << 20)) return fail(ARL_EINVAL, "stamps_begin: cap out of [1, 2^20]");
  arl::Net& n = h->net;
  if (!n.stamps) n.stamps = new arl::Stamps();
  arl::Stamps& st = *n.stamps;
  while ((int)st.ev.size() < cap) {
    hipEvent_t e;
    // timing events without the system-scope fence (cache writeback / invalidate) a default event
    // record performs: the stamps perturb the window they measure less
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess)
      return fail(ARL_EHIP, "stamps_begin: hipEventCreateWithFlags");
    st.ev.push_back(e);
  }
  st.stage.assign(st.ev.size(), 0);
  st.seq.assign(st.ev.size(), 0);
  st.count = 0;
  st.calls = 0;
  st.period = 0;
  st.on = true;
  return ARL_OK;
}

int arl_stamps_sparse(arl_net* h, int period) {
  NEED_BOUND(h);
  arl::Stamps* st = h->net.stamps;
  if (!st || !st->on || st->calls != 0) return fail(ARL_EINVAL, "stamps_sparse: call right after arl_stamps_begin");
  if (period < 0 || period > 4096) return fail(ARL_EINVAL, "stamps_sparse: period out of [0, 4096]");
  st->period = period;
  return ARL_OK;
}

int arl_stamp(arl_net* h, int stage, void* s) {
  NEED_BOUND(h);
  if (stage < 0 || stage > arl::STAGE_OTHER) return fail(ARL_EINVAL, "stamp: unknown stage");
  return hip_status(arl::stamp(h->net, stage, S(s)), "stamp");
}

int arl_stamps_end(arl_net* h, int* count) {
  NEED_BOUND(h);
  arl::Stamps* st = h->net.stamps;
  if (st) st->on = false;
  if (count) *count = st ? st->count : 0;
  return ARL_OK;
}

int arl_stamps_read(arl_net* h, int i0, int n, float* ms, int* stage) {
  NEED_BOUND(h);
  arl::Stamps* st = h->net.stamps;
  if (!st || i0 < 0 || n < 0 || i0 + n > st->count) return fail(ARL_EINVAL, "stamps_read: range outside the stamps");
  if (n == 0) return ARL_OK;
  if (!ms || !stage) return fail(ARL_EINVAL, "stamps_read: null output");
  hipError_t e = hipEventSynchronize(st->ev[i0 + n - 1]);
  for (int i = i0; i < i0 + n && e == hipSuccess; ++i) {
    float t = 0.f;
    if (i > 0 && st->seq[i] != st->seq[i - 1] + 1) t = -1.f;   // (sparse: not one stage's interval)
    else if (i > 0) e = hipEventElapsedTime(&t, st->ev[i - 1], st->ev[i]);
    ms[i - i0] = t;
    stage[i - i0] = st->stage[i];
  }
  return hip_status(e, "stamps_read");
}

int arl_learn(arl_net* h, double gamma, double beta, double vcoef, int clip_reward, void* s) {
  NEED_BOUND(h);
  return hip_status(arl::net_learn(h->net, gamma, (float)beta, (float)vcoef, clip_reward, S(s)), "learn");
}

int arl_learn_part(arl_net* h, int part, double gamma, double beta, double vcoef, int clip_reward, void* s) {
  NEED_BOUND(h);
  if (part < 0 || part >= arl::LEARN_PARTS) return fail(ARL_EINVAL, "learn_part: part out of range");
  if (h->net.arch == arl::ARCH_FF_NATURE) return fail(ARL_ESTATE, "learn_part: the Nature learner is one call");
  return hip_status(arl::net_learn_part(h->net, part, gamma, (float)beta, (float)vcoef, clip_reward, S(s)),
                    "learn_part");
}

int arl_optimize(arl_net* h, double lr0, int64_t total_steps, int64_t n_total, double alpha, double eps, double clip,
                 void* s) {
  NEED_BOUND(h);
  return hip_status(arl::net_optimize(h->net, lr0, total_steps, n_total, alpha, eps, (float)clip, S(s)), "optimize");
}

int arl_run_window(arl_net* h, const uint8_t* pair_pool, const float* reward_pool, const uint8_t* done_pool,
                   int64_t pool_len, int first, int resize_mode, double gamma, double beta, double vcoef,
                   int clip_reward, double lr0, int64_t total_steps, int64_t n_total, double alpha, double eps,
                   double clip, void* s) {
  NEED_BOUND(h);
  arl::Net& n = h->net;
  if (n.rgb || n.stack || n.states || n.arch == arl::ARCH_FF_NATURE)
    return fail(ARL_ESTATE, "run_window: frame-pair nets with the NIPS head only (FF / LSTM)");
  if (resize_mode < 0 || resize_mode > (ARL_RESIZE_SIMD | ARL_RESIZE_CROP)) return fail(ARL_EINVAL, "bad resize_mode");
  {   // every observation of the window reads the same pools: check them before the first launch
    arl::RingArgs a;
    if (int rc = ring_args(h, 0, pair_pool, reward_pool, done_pool, pool_len, 0, resize_mode, 0, 0, 0, -1, a)) return rc;
  }
  // FF: the learner's returns + heads backward run in the bootstrap step's policy launch
  const bool fuse_was = n.fuse_returns;
  const arl::Net::ReturnsCfg ret_was = n.ret;
  n.fuse_returns = n.arch == arl::ARCH_FF;
  n.returns_done = false;
  n.ret = arl::Net::ReturnsCfg{gamma, (float)beta, (float)vcoef, clip_reward};
  for (int t = 0; t <= n.T; ++t) {
    if (t > 0 || first) {   // slot 0 of a continuing window: the previous window's bootstrap observation
      const int rc = observe_common(h, t, pair_pool, reward_pool, done_pool, pool_len, t == 0 ? 1 : 0, resize_mode, 0,
                                    0, s);
      if (rc != ARL_OK) {
        n.fuse_returns = fuse_was;
        n.ret = ret_was;
        return rc;
      }
    }
    const hipError_t e = arl::net_act(n, t, 1, S(s));   // (slot T: the bootstrap forward, no draw)
    if (e != hipSuccess) {
      n.fuse_returns = fuse_was;
      n.ret = ret_was;
      return hip_status(e, "run_window: act");
    }
  }
  n.fuse_returns = fuse_was;
  n.ret = ret_was;
  hipError_t e = arl::net_learn(n, gamma, (float)beta, (float)vcoef, clip_reward, S(s));
  if (e == hipSuccess) e = arl::net_optimize(n, lr0, total_steps, n_total, alpha, eps, (float)clip, S(s), true);
  return hip_status(e, "run_window");
}

int arl_optimize_advance(arl_net* h, double lr0, int64_t total_steps, int64_t n_total, double alpha, double eps,
                         double clip, void* s) {
  NEED_BOUND(h);
  return hip_status(arl::net_optimize(h->net, lr0, total_steps, n_total, alpha, eps, (float)clip, S(s), true),
                    "optimize_advance");
}

int arl_advance(arl_net* h, void* s) {
  NEED_BOUND(h);
  return hip_status(arl::net_advance(h->net, S(s)), "advance");
}

int arl_forward_states(arl_net* h, const float* x, int64_t n, int mode, void* s) {
  NEED_BOUND(h);
  const bool keep = (mode & ARL_FWD_KEEP_STATE) != 0;
  mode &= ~ARL_FWD_KEEP_STATE;
  if (mode < 0 || mode > 2) return fail(ARL_EINVAL, "forward_states: mode must be 0, 1 or 2 (| ARL_FWD_KEEP_STATE)");
  if (!x || n < 1 || n > h->net.N) return fail(ARL_EINVAL, "forward_states: need 1 <= n <= n_envs");
  if (!aligned(x, 16)) return fail(ARL_EINVAL, "forward_states: states must be 16-byte aligned");
  return hip_status(arl::net_forward_f32(h->net, x, (int)n, mode, S(s), keep), "forward_states");
}

int arl_reset_state(arl_net* h, int64_t e0, int64_t n, void* s) {
  NEED_BOUND(h);
  if (e0 < 0 || n < 0 || e0 + n > h->net.N) return fail(ARL_EINVAL, "reset_state: rows outside [0, n_envs)");
  if (n == 0) return ARL_OK;
  return hip_status(arl::net_reset_state(h->net, (int)e0, (int)n, S(s)), "reset_state");
}

int arl_rmsprop(float* p, float* ms, const float* g, int64_t n, double lr, double alpha, double eps, double clip,
                double* parts, void* s) {
  if (n < 0 || (n > 0 && (!p || !ms || !g))) return fail(ARL_EINVAL, "rmsprop: null pointer / n < 0");
  if (!aligned(p, 16) || !aligned(ms, 16) || !aligned(g, 16)) return fail(ARL_EINVAL, "rmsprop: 16-byte alignment");
  if (clip > 0 && !parts) return fail(ARL_EINVAL, "rmsprop: clip needs norm_partials scratch");
  hipError_t e = hipSuccess;
  const int blocks = 256;
  if (clip > 0) e = arl::launch_grad_sqnorm(g, n, parts, blocks, S(s));
  if (e == hipSuccess)
    e = arl::launch_rmsprop(p, ms, g, n, lr, alpha, eps, clip > 0 ? parts : nullptr, blocks, (float)clip, nullptr, 0,
                            0, 0, S(s));
  return hip_status(e, "rmsprop");
}

int arl_policy(const float* hh, int64_t n, const float* Wpi, const float* bpi, const float* Wv, const float* bv,
               int A, uint64_t seed, const int64_t* step_dev, int64_t step_off, int env_offset, int sample,
               float* logits, float* probs, float* logp, float* v, float* ent, int32_t* act, float* logp_a,
               void* s) {
  if (n < 0 || A < 1 || A > arl::MAXA) return fail(ARL_EINVAL, "policy: bad n / n_actions");
  if (n > 0 && (!hh || !Wpi || !bpi || !Wv || !bv || !logits || !probs || !logp || !v || !ent))
    return fail(ARL_EINVAL, "policy: null pointer");
  if (sample < 0 || sample > 2) return fail(ARL_EINVAL, "policy: sample must be 0, 1 (Philox draw) or 2 (argmax)");
  if (sample == 1 && !step_dev) return fail(ARL_EINVAL, "policy: sampling needs the device step counter");
  if (sample && (!act || !logp_a)) return fail(ARL_EINVAL, "policy: sampling needs act/logp_a");
  if (!aligned(hh, 16) || !aligned(Wpi, 16) || !aligned(Wv, 16)) return fail(ARL_EINVAL, "policy: 16-byte alignment");
  return hip_status(arl::launch_policy(hh, n, Wpi, bpi, Wv, bv, A, seed, step_dev, step_off, env_offset, sample,
                                       logits, probs, logp, v, ent, act, logp_a, S(s)),
                    "policy");
}

int arl_returns_lossgrad(const float* rewards, const uint8_t* dones, const float* v, const float* probs,
                         const float* logp, const int32_t* act, int T, int64_t n, int A, double gamma, double beta,
                         double pi_loss_coef, double vcoef, int keep_loss_scale_same, int clip_reward, float* dlogits,
                         float* dv, float* loss, void* s) {
  if (T < 1 || n < 0 || A < 1) return fail(ARL_EINVAL, "returns: bad T / n / A");
  if (n > 0 && (!rewards || !dones || !v || !probs || !logp || !act || !dlogits || !dv))
    return fail(ARL_EINVAL, "returns: null pointer");
  return hip_status(arl::launch_returns(rewards, dones, v, probs, logp, act, T, (int)n, A, gamma, (float)beta,
                                        (float)vcoef, clip_reward, dlogits, dv, loss, S(s), nullptr,
                                        (float)pi_loss_coef, keep_loss_scale_same ? 1 : 0),
                    "returns");
}

int arl_stream_copy(const void* src, void* dst, int64_t bytes, int blocks, int mode, void* s) {
  if (bytes < 0 || (bytes > 0 && (!src || !dst))) return fail(ARL_EINVAL, "stream_copy: null pointer / bytes < 0");
  if (bytes % 16 || !aligned(src, 16) || !aligned(dst, 16)) return fail(ARL_EINVAL, "stream_copy: 16-byte units");
  if (mode < 0 || mode > 3) return fail(ARL_EINVAL, "stream_copy: mode must be 0, 1, 2 or 3");
  if (mode < 2 && (blocks < 1 || blocks > 65535)) return fail(ARL_EINVAL, "stream_copy: blocks out of [1, 65535]");
  if (bytes == 0) return ARL_OK;
  return hip_status(arl::launch_stream_copy(src, dst, bytes, blocks, mode, S(s)), "stream_copy");
}

}  // extern "C"
