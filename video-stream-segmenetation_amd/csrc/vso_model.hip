// vso_model.hip — ONNX sessions (include/vso.h): protobuf reader, shape
// inference and constant folding at create, a fixed launch list over
// preallocated HBM tensors at run time (captured once in a hipGraph).
//
// What it replaces: onnxruntime-web's InferenceSession as the reference uses
// it (client/src/core/model.ts:12-67; session.run at frameProcessorTest.ts:91,
// :406, :478), through the same kind of entry points as ORT-web's wasm
// exports (_OrtCreateSession / _OrtRun / _OrtGetLastError,
// client/public/ort-wasm-simd-threaded.mjs:50-53).
//
// Planning rules:
//  * every shape is static once input 0's shape is fixed; nodes whose inputs
//    are all constants (the exporters' Shape/Gather/Concat/... arithmetic,
//    weight reshapes) are evaluated on the host at create;
//  * Reshape / Flatten / Squeeze / Unsqueeze / Identity alias their input;
//  * Conv absorbs a following BatchNormalization (weights folded), residual
//    Add and activation (Relu, Clip, PRelu, LeakyRelu, Sigmoid, Tanh) into
//    one launch when each intermediate has exactly one consumer;
//  * every other runtime node is one launch (vso_kernels.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "../../include/vso.h"
#include "vso_kernels.h"

using namespace vso;

namespace {

thread_local std::string g_err;

enum { DT_FLOAT = 1, DT_UINT8 = 2, DT_INT8 = 3, DT_INT32 = 6, DT_INT64 = 7, DT_BOOL = 9, DT_FLOAT16 = 10,
       DT_DOUBLE = 11, DT_UINT4 = 21, DT_INT4 = 22 };

// ---- protobuf wire format ---------------------------------------------------
struct PB {
  const uint8_t* p;
  const uint8_t* e;
  bool bad = false;
  bool more() const { return !bad && p < e; }
  uint64_t varint() {
    uint64_t r = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= e) { bad = true; return 0; }
      const uint8_t c = *p++;
      r |= (uint64_t)(c & 0x7F) << s;
      if (c < 0x80) return r;
    }
    bad = true;
    return 0;
  }
  bool key(uint32_t& f, uint32_t& wt) {
    const uint64_t k = varint();
    f = (uint32_t)(k >> 3);
    wt = (uint32_t)(k & 7);
    return !bad;
  }
  PB sub() {
    const uint64_t n = varint();
    if (bad || n > (uint64_t)(e - p)) { bad = true; return PB{e, e}; }
    PB s{p, p + n};
    p += n;
    return s;
  }
  uint32_t fixed32() {
    if (e - p < 4) { bad = true; return 0; }
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  uint64_t fixed64() {
    if (e - p < 8) { bad = true; return 0; }
    uint64_t v;
    std::memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  std::string str() {
    PB s = sub();
    return std::string(reinterpret_cast<const char*>(s.p), s.e - s.p);
  }
  void skip(uint32_t wt) {
    if (wt == 0) varint();
    else if (wt == 1) fixed64();
    else if (wt == 2) sub();
    else if (wt == 5) fixed32();
    else bad = true;
  }
};

void read_int64s(PB& pb, uint32_t wt, std::vector<int64_t>& out) {
  if (wt == 2) {
    PB s = pb.sub();
    while (s.more()) out.push_back((int64_t)s.varint());
    pb.bad |= s.bad;
  } else {
    out.push_back((int64_t)pb.varint());
  }
}

void read_floats(PB& pb, uint32_t wt, std::vector<float>& out) {
  if (wt == 2) {
    PB s = pb.sub();
    while (s.more()) {
      const uint32_t u = s.fixed32();
      float f;
      std::memcpy(&f, &u, 4);
      out.push_back(f);
    }
    pb.bad |= s.bad;
  } else {
    const uint32_t u = pb.fixed32();
    float f;
    std::memcpy(&f, &u, 4);
    out.push_back(f);
  }
}

float half_to_float(uint16_t h) {
  const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 31, m = h & 1023;
  uint32_t u;
  if (e == 0) {
    if (m == 0) u = s;
    else {  // subnormal
      float f = std::ldexp((float)m, -24);
      std::memcpy(&u, &f, 4);
      u |= s;
    }
  } else if (e == 31) {
    u = s | 0x7F800000u | (m << 13);
  } else {
    u = s | ((e + 112) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// f -> the nearest float16 value (ties to even), as a float: what a Cast to
// FLOAT16 or a float16-typed result holds (the GPU's __float2half_rn).
// f -> bfloat16 bits, round to nearest even (NaN stays NaN)
uint16_t float_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// f -> float16 bits, round to nearest even (the GPU's __float2half_rn)
uint16_t float_to_half_bits(float f) {
  const _Float16 h = (_Float16)f;
  uint16_t b;
  std::memcpy(&b, &h, 2);
  return b;
}

float round_half(float f) {
  const float a = std::fabs(f);
  if (!(a < INFINITY)) return f;  // inf / nan
  float q;
  if (a >= 65520.f) q = INFINITY;
  else if (a < 6.103515625e-05f) q = std::nearbyint(a * 16777216.f) / 16777216.f;  // subnormal: quantum 2^-24
  else {
    int e = 0;
    (void)std::frexp(a, &e);  // a in [2^(e-1), 2^e): 11 significant bits
    const float sc = std::ldexp(1.f, 11 - e);
    q = std::nearbyint(a * sc) / sc;
  }
  return std::copysign(q, f);
}

// A constant tensor (initializer / attribute / folded value).
struct Const {
  std::vector<int64_t> dims;
  bool is_int = false;
  bool f16 = false;        // float16-typed (values are exact halves)
  std::vector<float> f;    // float data (also filled for ints, as doubles would be)
  std::vector<int64_t> i;  // integer data
  int64_t numel() const {
    int64_t n = 1;
    for (int64_t d : dims) n *= d;
    return n;
  }
};

bool parse_tensor(PB pb, std::string* name, Const* c, std::string* err) {
  int dt = DT_FLOAT;
  std::string raw;
  bool has_raw = false;
  std::vector<float> fl;
  std::vector<int64_t> i32, i64;
  std::vector<double> dbl;
  uint32_t f, wt;
  while (pb.more() && pb.key(f, wt)) {
    if (f == 1) read_int64s(pb, wt, c->dims);
    else if (f == 2) dt = (int)pb.varint();
    else if (f == 4) read_floats(pb, wt, fl);
    else if (f == 5) read_int64s(pb, wt, i32);
    else if (f == 7) read_int64s(pb, wt, i64);
    else if (f == 8) *name = pb.str();
    else if (f == 9) { raw = pb.str(); has_raw = true; }
    else if (f == 10) {
      if (wt == 2) {
        PB s = pb.sub();
        while (s.more()) { const uint64_t u = s.fixed64(); double d; std::memcpy(&d, &u, 8); dbl.push_back(d); }
      } else { const uint64_t u = pb.fixed64(); double d; std::memcpy(&d, &u, 8); dbl.push_back(d); }
    } else if (f == 14) {
      if (pb.varint() == 1) { *err = "external tensor data is not supported"; return false; }
    } else pb.skip(wt);
  }
  if (pb.bad) { *err = "malformed TensorProto"; return false; }
  const int64_t n = c->numel();
  auto set_ints = [&](const std::vector<int64_t>& v) {
    c->is_int = true;
    c->i = v;
    c->f.assign(v.begin(), v.end());
  };
  switch (dt) {
    case DT_FLOAT:
      if (has_raw) { c->f.resize(raw.size() / 4); std::memcpy(c->f.data(), raw.data(), c->f.size() * 4); }
      else c->f = fl;
      break;
    case DT_FLOAT16: {
      std::vector<uint16_t> h;
      if (has_raw) { h.resize(raw.size() / 2); std::memcpy(h.data(), raw.data(), h.size() * 2); }
      else for (int64_t v : i32) h.push_back((uint16_t)v);
      for (uint16_t v : h) c->f.push_back(half_to_float(v));
      c->f16 = true;
      break;
    }
    case DT_UINT4: case DT_INT4: {  // two per byte, low nibble first
      std::vector<int64_t> v;
      const std::string& src = has_raw ? raw : std::string();
      for (int64_t k = 0; k < n; ++k) {
        int q = 0;
        if (has_raw) {
          if ((size_t)(k / 2) >= src.size()) break;
          q = ((uint8_t)src[k / 2] >> ((k & 1) * 4)) & 15;
        } else {
          if ((size_t)(k / 2) >= i32.size()) break;
          q = ((int)i32[k / 2] >> ((k & 1) * 4)) & 15;
        }
        v.push_back(dt == DT_INT4 && q >= 8 ? q - 16 : q);
      }
      set_ints(v);
      break;
    }
    case DT_DOUBLE:
      if (has_raw) { dbl.resize(raw.size() / 8); std::memcpy(dbl.data(), raw.data(), dbl.size() * 8); }
      c->f.assign(dbl.begin(), dbl.end());
      break;
    case DT_INT64:
      if (has_raw) { std::vector<int64_t> v(raw.size() / 8); std::memcpy(v.data(), raw.data(), v.size() * 8); set_ints(v); }
      else set_ints(i64);
      break;
    case DT_INT32: case DT_INT8: case DT_UINT8: case DT_BOOL: {
      std::vector<int64_t> v;
      if (has_raw) {
        const size_t es = dt == DT_INT32 ? 4 : 1;
        for (size_t k = 0; k + es <= raw.size(); k += es) {
          if (dt == DT_INT32) { int32_t x; std::memcpy(&x, raw.data() + k, 4); v.push_back(x); }
          else if (dt == DT_INT8) v.push_back((int8_t)raw[k]);
          else v.push_back((uint8_t)raw[k]);
        }
      } else v = i32;
      set_ints(v);
      break;
    }
    default:
      *err = "tensor data type " + std::to_string(dt) + " is not supported";
      return false;
  }
  if ((int64_t)c->f.size() != n) { *err = "tensor '" + *name + "' size does not match its dims"; return false; }
  return true;
}

struct Attr {
  bool has_f = false, has_i = false, has_s = false, has_t = false;
  float f = 0.f;
  int64_t i = 0;
  std::string s;
  std::vector<float> fs;
  std::vector<int64_t> is;
  Const t;
};

struct Node {
  std::string op, name;
  std::vector<std::string> in, out;
  std::map<std::string, Attr> attrs;
  int64_t ai(const char* k, int64_t d) const {
    auto it = attrs.find(k);
    return it != attrs.end() && it->second.has_i ? it->second.i : d;
  }
  float af(const char* k, float d) const {
    auto it = attrs.find(k);
    return it != attrs.end() && it->second.has_f ? it->second.f : d;
  }
  std::string as(const char* k, const char* d) const {
    auto it = attrs.find(k);
    return it != attrs.end() && it->second.has_s ? it->second.s : std::string(d);
  }
  bool has(const char* k) const { return attrs.count(k) != 0; }
  std::vector<int64_t> ais(const char* k) const {
    auto it = attrs.find(k);
    return it != attrs.end() ? it->second.is : std::vector<int64_t>{};
  }
};

bool parse_attr(PB pb, std::string* name, Attr* a, std::string* err) {
  uint32_t f, wt;
  while (pb.more() && pb.key(f, wt)) {
    if (f == 1) *name = pb.str();
    else if (f == 2) { const uint32_t u = pb.fixed32(); std::memcpy(&a->f, &u, 4); a->has_f = true; }
    else if (f == 3) { a->i = (int64_t)pb.varint(); a->has_i = true; }
    else if (f == 4) { a->s = pb.str(); a->has_s = true; }
    else if (f == 5) { std::string tn; if (!parse_tensor(pb.sub(), &tn, &a->t, err)) return false; a->has_t = true; }
    else if (f == 7) read_floats(pb, wt, a->fs);
    else if (f == 8) read_int64s(pb, wt, a->is);
    else pb.skip(wt);
  }
  if (pb.bad) { *err = "malformed AttributeProto"; return false; }
  return true;
}

struct IO {
  std::string name;
  std::vector<int64_t> dims;  // -1 = symbolic
};

bool parse_value_info(PB pb, IO* io) {
  uint32_t f, wt;
  while (pb.more() && pb.key(f, wt)) {
    if (f == 1) io->name = pb.str();
    else if (f == 2) {
      PB tp = pb.sub();
      uint32_t f2, w2;
      while (tp.more() && tp.key(f2, w2)) {
        if (f2 != 1) { tp.skip(w2); continue; }
        PB tt = tp.sub();
        uint32_t f3, w3;
        while (tt.more() && tt.key(f3, w3)) {
          if (f3 != 2) { tt.skip(w3); continue; }
          PB sh = tt.sub();
          uint32_t f4, w4;
          while (sh.more() && sh.key(f4, w4)) {
            if (f4 != 1) { sh.skip(w4); continue; }
            PB dm = sh.sub();
            int64_t d = -1;
            uint32_t f5, w5;
            while (dm.more() && dm.key(f5, w5)) {
              if (f5 == 1) d = (int64_t)dm.varint();
              else dm.skip(w5);
            }
            io->dims.push_back(d);
          }
        }
      }
    } else pb.skip(wt);
  }
  return !pb.bad;
}

struct Graph {
  std::vector<Node> nodes;
  std::map<std::string, Const> inits;
  std::vector<IO> inputs, outputs;
};

bool parse_model(const uint8_t* data, size_t n, Graph* g, std::string* err) {
  PB m{data, data + n};
  uint32_t f, wt;
  bool have_graph = false;
  while (m.more() && m.key(f, wt)) {
    if (f != 7) { m.skip(wt); continue; }
    have_graph = true;
    PB gp = m.sub();
    uint32_t f2, w2;
    while (gp.more() && gp.key(f2, w2)) {
      if (f2 == 1) {
        PB np = gp.sub();
        Node nd;
        uint32_t f3, w3;
        while (np.more() && np.key(f3, w3)) {
          if (f3 == 1) nd.in.push_back(np.str());
          else if (f3 == 2) nd.out.push_back(np.str());
          else if (f3 == 3) nd.name = np.str();
          else if (f3 == 4) nd.op = np.str();
          else if (f3 == 5) {
            std::string an;
            Attr a;
            if (!parse_attr(np.sub(), &an, &a, err)) return false;
            nd.attrs[an] = a;
          } else np.skip(w3);
        }
        if (np.bad) { *err = "malformed NodeProto"; return false; }
        g->nodes.push_back(nd);
      } else if (f2 == 5) {
        std::string tn;
        Const c;
        if (!parse_tensor(gp.sub(), &tn, &c, err)) return false;
        g->inits[tn] = c;
      } else if (f2 == 11 || f2 == 12) {
        IO io;
        if (!parse_value_info(gp.sub(), &io)) { *err = "malformed ValueInfoProto"; return false; }
        (f2 == 11 ? g->inputs : g->outputs).push_back(io);
      } else gp.skip(w2);
    }
    if (gp.bad) { *err = "malformed GraphProto"; return false; }
  }
  if (m.bad || !have_graph) { *err = "not an ONNX ModelProto (no graph)"; return false; }
  // graph inputs that are initializers are constants, not feeds
  std::vector<IO> feeds;
  for (const IO& io : g->inputs)
    if (!g->inits.count(io.name)) feeds.push_back(io);
  g->inputs = feeds;
  return true;
}

}  // namespace

// ---- the session -----------------------------------------------------------
struct Value {
  std::vector<int64_t> shape;
  bool is_const = false;
  Const c;          // when is_const
  int buf = -1;     // runtime tensor: device buffer id
  int64_t numel() const {
    int64_t n = 1;
    for (int64_t d : shape) n *= d;
    return n;
  }
};

// A host region holding a launch's parameters: at capture, every aligned
// 8-byte word of it that points into one of the session's device
// allocations marks that allocation as used by the launch (read or written:
// the lane schedule treats every use as a conflict).
struct Region {
  std::shared_ptr<const void> keep;
  const void* p;
  size_t n;
};

struct Launch {
  std::string name;
  std::function<void(hipStream_t)> fn;
  std::vector<Region> io;
};

struct DevRange {
  uintptr_t lo, hi;
  bool ro;  // constants: never written by a kernel (no dependency through them)
};

struct vso_session {
  int device = 0;
  int conv_precision = 0;  // ConvPrec
  int tile_convs = 0;      // convolutions planned on k_conv_tile
  int ir_blocks = 0;       // inverted residual blocks planned on k_ir
  hipStream_t stream = nullptr;
  std::string err;
  std::vector<std::string> in_names, out_names;
  std::vector<std::vector<int64_t>> in_shapes, out_shapes;
  std::vector<float*> bufs;
  std::vector<int64_t> buf_elems;
  std::vector<int> in_bufs, out_bufs;
  std::vector<void*> allocs;
  std::vector<Launch> launches;
  std::vector<DevRange> ranges;   // every device allocation of the session
  hipStream_t side = nullptr;     // the second capture lane
  std::vector<hipEvent_t> events; // cross-lane edges of the captured graph
  int lanes_used = 1;             // lanes of the captured schedule (vso_lane_count)
  hipGraphExec_t graph = nullptr;
  std::atomic<int> busy{0};
};

namespace {

struct Planner {
  vso_session* s;
  Graph& g;
  std::map<std::string, Value> vals;
  std::map<std::string, int> consumers;
  std::set<size_t> done;  // node indices absorbed by a fused launch
  // Add operands computed inside the consuming convolution's epilogue instead
  // of by their own launches: MaxPool(2x2, s2) -> [Pad of the channel axis] -> Add
  struct ResFuse {
    std::string src;  // the MaxPool's input, or the Pad's input
    int mode;         // Epilogue::res_mode
  };
  std::map<std::string, ResFuse> res_fuse;
  std::map<std::string, std::pair<const float*, DwPre>> pending_dw;  // dw outputs computed in their 1x1 consumer (input, producer)
  std::map<const void*, float*> dev_consts;
  // Concat (axis 1) inputs whose producer — a convolution or a Resize — writes
  // them straight into the concatenation (find_concat_direct): value name ->
  // patches re-pointing the producing launches' output there, applied when the
  // Concat is planned (base: the input's first channel of image 0; ctot: the
  // concatenation's channels), which then copies only the other inputs.
  // MODNet: 10 of its 13 Concat copies (the k_copy_rows launches).
  std::set<std::string> cat_direct;
  // 2x linear Resizes computed inside their consumer convolution
  // (k_conv_tile_up): candidates by graph structure (find_up_fusions); the
  // planned ones not yet launched, by output name; and per Concat output, its
  // pending inputs' channel ranges.  A consumer that cannot take one launches
  // it just before itself (flush_up).
  std::set<std::string> up_cand;
  // InstanceNorm apply steps left to their consumer (k_conv_thin), by value name
  std::map<std::string, std::shared_ptr<NormParams>> norm_pending;
  std::map<std::string, std::shared_ptr<ResizeParams>> up_pending;
  struct UpRange { std::string name; int c0, c1; };
  std::map<std::string, std::vector<UpRange>> cat_up;
  std::map<std::string, std::vector<std::function<void(float*, int)>>> cat_patch;
  // A Concat's last input (whole 32-channel chunks on) left in its own tensor
  // instead of copied in: its sole consumer, a convolution on k_conv_tile,
  // reads those chunks from there (ConvTileParams::x2); any other plan runs
  // the copy just before itself (flush_tail).  MODNet: 3 copies of 8 x 3 /
  // 32 x H x W planes (52 us of k_copy_rows at batch 8).
  struct CatTail {
    const float* x;
    int c0, C;
    std::function<bool()> copy;
  };
  std::map<std::string, CatTail> cat_tail;
  std::string err;

  bool fail(const std::string& m) {
    err = m;
    return false;
  }

  template <class T>
  bool dalloc(T** p, size_t bytes) {
    void* q = nullptr;
    const size_t n = std::max<size_t>(bytes, 16);
    if (hipMalloc(&q, n) != hipSuccess) return fail("hipMalloc failed");
    s->allocs.push_back(q);
    s->ranges.push_back(DevRange{(uintptr_t)q, (uintptr_t)q + n, false});
    *p = static_cast<T*>(q);
    return true;
  }
  // a constant's allocation (weights, biases, tables): kernels only read it
  void mark_ro(const void* q) {
    for (DevRange& r : s->ranges)
      if ((uintptr_t)q >= r.lo && (uintptr_t)q < r.hi) r.ro = true;
  }
  template <class T>
  static Region reg(const std::shared_ptr<T>& sp) {
    return Region{std::static_pointer_cast<const void>(sp), sp.get(), sizeof(T)};
  }

  int new_buf(int64_t elems) {
    float* d = nullptr;
    if (!dalloc(&d, (size_t)std::max<int64_t>(elems, 1) * 4)) return -1;
    s->bufs.push_back(d);
    s->buf_elems.push_back(elems);
    return (int)s->bufs.size() - 1;
  }

  // device copy of a constant's float data (cached per Const)
  const float* upload(const Const& c) {
    auto it = dev_consts.find(&c);
    if (it != dev_consts.end()) return it->second;
    float* d = nullptr;
    if (!dalloc(&d, c.f.size() * 4)) return nullptr;
    if (!c.f.empty() && hipMemcpy(d, c.f.data(), c.f.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
      fail("constant upload failed");
      return nullptr;
    }
    dev_consts[&c] = d;
    mark_ro(d);
    return d;
  }
  const float* upload_vec(const std::vector<float>& v) {
    float* d = nullptr;
    if (!dalloc(&d, v.size() * 4)) return nullptr;
    if (!v.empty() && hipMemcpy(d, v.data(), v.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
      fail("constant upload failed");
      return nullptr;
    }
    mark_ro(d);
    return d;
  }

  Value* val(const std::string& n) {
    if (n.empty()) return nullptr;
    auto it = vals.find(n);
    return it == vals.end() ? nullptr : &it->second;
  }
  float* dptr(const Value& v) { return s->bufs[v.buf]; }
  // a runtime pointer for an operand: its buffer, or its uploaded constant
  const float* operand(Value& v) { return v.is_const ? upload(v.c) : s->bufs[v.buf]; }

  bool set_runtime(const std::string& name, const std::vector<int64_t>& shape, int alias = -1) {
    Value v;
    v.shape = shape;
    v.buf = alias >= 0 ? alias : new_buf(v.numel());
    if (v.buf < 0) return false;
    vals[name] = v;
    return true;
  }
  void set_const(const std::string& name, const Const& c) {
    Value v;
    v.is_const = true;
    v.c = c;
    v.shape = c.dims;
    vals[name] = v;
  }

  void add(const char* name, std::function<void(hipStream_t)> fn, std::vector<Region> io) {
    s->launches.push_back(Launch{name, fn, std::move(io)});
  }

  // ---- constant folding (host) ---------------------------------------------
  bool fold(const Node& nd, std::vector<Value*>& in) {
    const std::string& op = nd.op;
    Const r;
    auto ints = [](const Const& c) { return c.is_int ? c.i : std::vector<int64_t>(c.f.begin(), c.f.end()); };
    if (op == "Constant") {
      auto it = nd.attrs.find("value");
      if (it != nd.attrs.end() && it->second.has_t) r = it->second.t;
      else if (nd.has("value_float")) { r.f = {nd.af("value_float", 0)}; }
      else if (nd.has("value_int")) { r.is_int = true; r.i = {nd.ai("value_int", 0)}; r.f = {(float)r.i[0]}; }
      else if (nd.has("value_ints")) { r.is_int = true; r.i = nd.ais("value_ints"); r.dims = {(int64_t)r.i.size()}; r.f.assign(r.i.begin(), r.i.end()); }
      else if (nd.has("value_floats")) { r.f = nd.attrs.at("value_floats").fs; r.dims = {(int64_t)r.f.size()}; }
      else return fail("Constant without a supported value");
    } else if (op == "Shape") {
      r.is_int = true;
      r.i = in[0]->shape;
      int64_t st = nd.ai("start", 0), en = nd.ai("end", (int64_t)r.i.size());
      const int64_t rk = (int64_t)r.i.size();
      if (st < 0) st += rk;
      if (en < 0) en += rk;
      st = std::clamp<int64_t>(st, 0, rk);
      en = std::clamp<int64_t>(en, 0, rk);
      r.i = std::vector<int64_t>(r.i.begin() + st, r.i.begin() + std::max(st, en));
      r.dims = {(int64_t)r.i.size()};
      r.f.assign(r.i.begin(), r.i.end());
    } else if (op == "ConstantOfShape") {
      r.dims = ints(in[0]->c);
      float v = 0.f;
      bool is_int = false;
      auto it = nd.attrs.find("value");
      if (it != nd.attrs.end() && it->second.has_t && !it->second.t.f.empty()) {
        v = it->second.t.f[0];
        is_int = it->second.t.is_int;
      }
      r.is_int = is_int;
      r.f.assign((size_t)r.numel(), v);
      if (is_int) r.i.assign((size_t)r.numel(), (int64_t)v);
    } else if (op == "Identity" || op == "Cast" || op == "Floor" || op == "Ceil") {
      r = in[0]->c;
      if (op == "Cast") {
        const int64_t to = nd.ai("to", DT_FLOAT);
        const bool to_int = to == DT_INT64 || to == DT_INT32 || to == DT_INT8 || to == DT_UINT8 || to == DT_BOOL;
        if (to_int && !r.is_int) { r.i.clear(); for (float x : r.f) r.i.push_back((int64_t)x); }
        r.is_int = to_int;
        r.f16 = to == DT_FLOAT16;
        if (r.f16)
          for (float& x : r.f) x = round_half(x);
      } else if (op == "Floor" || op == "Ceil") {
        for (float& x : r.f) x = op == "Floor" ? std::floor(x) : std::ceil(x);
      }
    } else if (op == "Add" || op == "Sub" || op == "Mul" || op == "Div") {
      const Const &a = in[0]->c, &b = in[1]->c;
      const bool both_int = a.is_int && b.is_int;
      // broadcasting on small constant tensors
      const size_t ra = a.dims.size(), rb = b.dims.size(), rk = std::max(ra, rb);
      r.dims.assign(rk, 1);
      for (size_t d = 0; d < rk; ++d) {
        const int64_t da = d + ra >= rk ? a.dims[d + ra - rk] : 1, db = d + rb >= rk ? b.dims[d + rb - rk] : 1;
        if (da != db && da != 1 && db != 1) return fail(nd.op + ": incompatible constant shapes");
        r.dims[d] = std::max(da, db);
      }
      const int64_t n = r.numel();
      r.is_int = both_int;
      for (int64_t k = 0; k < n; ++k) {
        int64_t ka = 0, kb = 0, rem = k, sa = 1, sb = 1;
        for (int d = (int)rk - 1; d >= 0; --d) {
          const int64_t id = rem % r.dims[d];
          rem /= r.dims[d];
          const int64_t da = d + (int)ra >= (int)rk ? a.dims[d + ra - rk] : 1;
          const int64_t db = d + (int)rb >= (int)rk ? b.dims[d + rb - rk] : 1;
          if (da > 1) ka += id * sa;
          if (db > 1) kb += id * sb;
          sa *= da;
          sb *= db;
        }
        if (both_int) {
          const int64_t x = a.i[ka], y = b.i[kb];
          int64_t v = op == "Add" ? x + y : op == "Sub" ? x - y : op == "Mul" ? x * y
                                                                       : (y ? (int64_t)std::floor((double)x / y) : 0);
          r.i.push_back(v);
          r.f.push_back((float)v);
        } else {
          const double x = a.f[ka], y = b.f[kb];
          r.f.push_back((float)(op == "Add" ? x + y : op == "Sub" ? x - y : op == "Mul" ? x * y : x / y));
        }
      }
    } else if (op == "DequantizeLinear") {
      // y = (x - zero_point) * scale: per tensor, per axis, or blocked along
      // the axis (opset 21 block_size); int8/uint8/int4/uint4 weights
      const Const& x = in[0]->c;
      const Const& sc = in[1]->c;
      const Const* zp = in.size() > 2 && in[2] ? &in[2]->c : nullptr;
      if (!x.is_int) return fail("DequantizeLinear: integer input expected");
      const int64_t rk = (int64_t)x.dims.size();
      int64_t ax = nd.ai("axis", 1);
      if (ax < 0) ax += rk;
      const int64_t bs = nd.ai("block_size", 0);
      const int64_t n = x.numel(), ns = sc.numel();
      int64_t inner = 1;
      for (int64_t k = ax + 1; k < rk; ++k) inner *= x.dims[k];
      const int64_t da = rk > 0 && ax < rk ? x.dims[ax] : 1;
      const int64_t sda = bs > 0 && ax < (int64_t)sc.dims.size() ? sc.dims[ax] : 1;
      if (ns != 1 && (ax < 0 || ax >= rk)) return fail("DequantizeLinear: bad axis");
      if (ns != 1 && bs == 0 && ns != da) return fail("DequantizeLinear: per-axis scale size mismatch");
      if (bs > 0 && (sda != (da + bs - 1) / bs || ns != n / da * sda))
        return fail("DequantizeLinear: blocked scale shape mismatch");
      if (zp && zp->numel() != ns) return fail("DequantizeLinear: zero point shape differs from the scale's");
      r.dims = x.dims;
      r.f.resize((size_t)n);
      for (int64_t k = 0; k < n; ++k) {
        int64_t si = 0;
        if (ns != 1) {
          const int64_t ia = (k / inner) % da;
          if (bs == 0) si = ia;
          else si = ((k / (inner * da)) * sda + ia / bs) * inner + k % inner;
        }
        const double q = (double)x.i[k] - (zp ? (double)zp->i[si] : 0.0);
        float v = (float)(q * (double)sc.f[si]);
        if (sc.f16) v = round_half(v);
        r.f[k] = v;
      }
      r.f16 = sc.f16;
    } else if (op == "Gather") {
      const Const &d = in[0]->c, &ix = in[1]->c;
      int64_t ax = nd.ai("axis", 0);
      const int64_t rk = (int64_t)d.dims.size();
      if (ax < 0) ax += rk;
      int64_t outer = 1, inner = 1;
      for (int64_t k = 0; k < ax; ++k) outer *= d.dims[k];
      for (int64_t k = ax + 1; k < rk; ++k) inner *= d.dims[k];
      const std::vector<int64_t> idx = ints(ix);
      for (int64_t k = 0; k < ax; ++k) r.dims.push_back(d.dims[k]);
      for (int64_t v : ix.dims) r.dims.push_back(v);
      for (int64_t k = ax + 1; k < rk; ++k) r.dims.push_back(d.dims[k]);
      r.is_int = d.is_int;
      for (int64_t o = 0; o < outer; ++o)
        for (int64_t j : idx) {
          const int64_t jj = j < 0 ? j + d.dims[ax] : j;
          for (int64_t q = 0; q < inner; ++q) {
            const int64_t src = (o * d.dims[ax] + jj) * inner + q;
            r.f.push_back(d.f[src]);
            if (d.is_int) r.i.push_back(d.i[src]);
          }
        }
    } else if (op == "Unsqueeze" || op == "Squeeze" || op == "Reshape" || op == "Flatten") {
      r = in[0]->c;
      std::vector<int64_t> shp;
      if (!infer_view(nd, in, &shp)) return false;
      r.dims = shp;
    } else if (op == "Concat") {
      int64_t ax = nd.ai("axis", 0);
      const int64_t rk = (int64_t)in[0]->c.dims.size();
      if (ax < 0) ax += rk;
      r.dims = in[0]->c.dims;
      r.dims[ax] = 0;
      bool all_int = true;
      for (Value* v : in) { r.dims[ax] += v->c.dims[ax]; all_int = all_int && v->c.is_int; }
      int64_t outer = 1;
      for (int64_t k = 0; k < ax; ++k) outer *= r.dims[k];
      r.is_int = all_int;
      for (int64_t o = 0; o < outer; ++o)
        for (Value* v : in) {
          const int64_t blk = v->c.numel() / std::max<int64_t>(outer, 1);
          for (int64_t q = 0; q < blk; ++q) {
            r.f.push_back(v->c.f[o * blk + q]);
            if (all_int) r.i.push_back(v->c.i[o * blk + q]);
          }
        }
    } else if (op == "Slice") {
      const Const& d = in[0]->c;
      if (d.dims.size() != 1) return fail("Slice of a constant: rank 1 only");
      const std::vector<int64_t> st = ints(in[1]->c), en = ints(in[2]->c);
      const std::vector<int64_t> stp = in.size() > 4 && in[4] ? ints(in[4]->c) : std::vector<int64_t>{1};
      const int64_t L = d.dims[0];
      int64_t a = st[0] < 0 ? st[0] + L : st[0], b = en[0] < 0 ? en[0] + L : en[0];
      const int64_t step = stp[0];
      a = std::clamp<int64_t>(a, 0, L);
      b = std::clamp<int64_t>(b, step > 0 ? 0 : -1, L);
      r.is_int = d.is_int;
      for (int64_t k = a; step > 0 ? k < b : k > b; k += step) {
        r.f.push_back(d.f[k]);
        if (d.is_int) r.i.push_back(d.i[k]);
      }
      r.dims = {(int64_t)r.f.size()};
    } else if (op == "Transpose") {
      const Const& d = in[0]->c;
      std::vector<int64_t> perm = nd.ais("perm");
      const size_t rk = d.dims.size();
      if (perm.empty()) for (size_t k = 0; k < rk; ++k) perm.push_back((int64_t)(rk - 1 - k));
      r.dims.resize(rk);
      for (size_t k = 0; k < rk; ++k) r.dims[k] = d.dims[perm[k]];
      std::vector<int64_t> st(rk, 1);
      for (int k = (int)rk - 2; k >= 0; --k) st[k] = st[k + 1] * d.dims[k + 1];
      const int64_t n = r.numel();
      r.is_int = d.is_int;
      for (int64_t o = 0; o < n; ++o) {
        int64_t rem = o, src = 0;
        for (int k = (int)rk - 1; k >= 0; --k) {
          src += (rem % r.dims[k]) * st[perm[k]];
          rem /= r.dims[k];
        }
        r.f.push_back(d.f[src]);
        if (d.is_int) r.i.push_back(d.i[src]);
      }
    } else {
      return fail("cannot evaluate constant " + op + " (node '" + nd.name + "')");
    }
    if (r.f.size() != (size_t)r.numel()) return fail("constant " + op + " produced a malformed tensor");
    set_const(nd.out[0], r);
    return true;
  }

  // Output shape of the view ops (Reshape, Flatten, Squeeze, Unsqueeze).
  bool infer_view(const Node& nd, std::vector<Value*>& in, std::vector<int64_t>* out) {
    const std::vector<int64_t>& x = in[0]->shape;
    const int64_t rk = (int64_t)x.size();
    auto axes_of = [&](int64_t out_rank) -> std::vector<int64_t> {
      std::vector<int64_t> a = nd.ais("axes");
      if (a.empty() && in.size() > 1 && in[1]) {
        const Const& c = in[1]->c;
        a = c.is_int ? c.i : std::vector<int64_t>(c.f.begin(), c.f.end());
      }
      for (int64_t& v : a) if (v < 0) v += out_rank;
      std::sort(a.begin(), a.end());
      return a;
    };
    if (nd.op == "Reshape") {
      if (in.size() < 2 || !in[1] || !in[1]->is_const) return fail("Reshape needs a constant shape");
      const Const& c = in[1]->c;
      std::vector<int64_t> shp = c.is_int ? c.i : std::vector<int64_t>(c.f.begin(), c.f.end());
      const bool allowzero = nd.ai("allowzero", 0) != 0;
      int64_t known = 1, neg = -1;
      for (size_t k = 0; k < shp.size(); ++k) {
        if (shp[k] == 0 && !allowzero) shp[k] = k < x.size() ? x[k] : 1;
        if (shp[k] == -1) neg = (int64_t)k;
        else known *= shp[k];
      }
      int64_t total = 1;
      for (int64_t d : x) total *= d;
      if (neg >= 0) shp[neg] = known ? total / known : 0;
      *out = shp;
    } else if (nd.op == "Flatten") {
      int64_t ax = nd.ai("axis", 1);
      if (ax < 0) ax += rk;
      int64_t a = 1, b = 1;
      for (int64_t k = 0; k < rk; ++k) (k < ax ? a : b) *= x[k];
      *out = {a, b};
    } else if (nd.op == "Squeeze") {
      std::vector<int64_t> axes = axes_of(rk);
      out->clear();
      for (int64_t k = 0; k < rk; ++k) {
        const bool drop = axes.empty() ? x[k] == 1 : std::binary_search(axes.begin(), axes.end(), k);
        if (!drop) out->push_back(x[k]);
      }
    } else {  // Unsqueeze
      std::vector<int64_t> a0 = nd.ais("axes");
      if (a0.empty() && in.size() > 1 && in[1]) a0 = in[1]->c.is_int ? in[1]->c.i : std::vector<int64_t>{};
      const int64_t orank = rk + (int64_t)a0.size();
      std::vector<int64_t> axes = axes_of(orank);
      out->clear();
      size_t j = 0;
      for (int64_t k = 0; k < orank; ++k) {
        if (std::binary_search(axes.begin(), axes.end(), k)) out->push_back(1);
        else out->push_back(x[j++]);
      }
    }
    int64_t a = 1, b = 1;
    for (int64_t d : x) a *= d;
    for (int64_t d : *out) b *= d;
    if (a != b) return fail(nd.op + " '" + nd.name + "': element count changes");
    return true;
  }

  // ---- runtime ops ---------------------------------------------------------
  static bool is_act(const std::string& op) {
    return op == "Relu" || op == "Clip" || op == "PRelu" || op == "LeakyRelu" || op == "Sigmoid" || op == "Tanh";
  }

  // the single node consuming `name`, if exactly one and `name` is no graph output
  int sole_consumer(const std::string& name, size_t after) {
    if (consumers[name] != 1) return -1;
    for (const IO& o : g.outputs)
      if (o.name == name) return -1;
    for (size_t k = after + 1; k < g.nodes.size(); ++k)
      for (const std::string& i : g.nodes[k].in)
        if (i == name) return (int)k;
    return -1;
  }

  // activation parameters of an activation node (constants only)
  bool act_of(const Node& nd, Epilogue* ep, int channels) {
    if (nd.op == "Relu") ep->act = ACT_RELU;
    else if (nd.op == "Sigmoid") ep->act = ACT_SIGMOID;
    else if (nd.op == "Tanh") ep->act = ACT_TANH;
    else if (nd.op == "LeakyRelu") { ep->act = ACT_LEAKY; ep->a0 = nd.af("alpha", 0.01f); }
    else if (nd.op == "Clip") {
      float lo = nd.af("min", -INFINITY), hi = nd.af("max", INFINITY);
      if (nd.in.size() > 1 && !nd.in[1].empty()) { Value* v = val(nd.in[1]); if (!v || !v->is_const) return false; lo = v->c.f[0]; }
      if (nd.in.size() > 2 && !nd.in[2].empty()) { Value* v = val(nd.in[2]); if (!v || !v->is_const) return false; hi = v->c.f[0]; }
      ep->act = ACT_CLIP; ep->a0 = lo; ep->a1 = hi;
    } else if (nd.op == "PRelu") {
      Value* sl = val(nd.in[1]);
      if (!sl || !sl->is_const) return false;
      const int64_t n = sl->c.numel();
      if (n != 1 && n != channels) return false;
      // slope must vary along the channel axis only ([C], [C,1,1], [1,C,1,1], or one value)
      int nontriv = 0;
      for (int64_t d : sl->c.dims) nontriv += d > 1;
      if (nontriv > 1) return false;
      ep->act = ACT_PRELU;
      ep->slope = upload(sl->c);
      ep->slope_stride = n == 1 ? 0 : 1;
    } else return false;
    return true;
  }


  // VSO_CAT_TAIL=0: every Concat input not written in place is copied (A/B knob)
  static bool cat_tail_enabled() {
    static const bool on = [] {
      const char* e = std::getenv("VSO_CAT_TAIL");
      return !(e && e[0] == '0');
    }();
    return on;
  }

  // VSO_GEMM_ACT=0: a Gemm / MatMul's activation as its own launch (A/B knob)
  static bool gemm_act_enabled() {
    static const bool on = [] {
      const char* e = std::getenv("VSO_GEMM_ACT");
      return !(e && e[0] == '0');
    }();
    return on;
  }

  // VSO_IR=0: the inverted residual blocks as three launches each (A/B knob)
  static bool ir_enabled() {
    static const bool on = [] {
      const char* e = std::getenv("VSO_IR");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  // the bf16x3 form in bf16 / f16 sessions (VSO_IR_B16=0: the f32 form there too)
  static bool ir_b16_enabled() {
    static const bool on = [] {
      const char* e = std::getenv("VSO_IR_B16");
      return !(e && e[0] == '0');
    }();
    return on;
  }

  // A constant conv's geometry: 1x1 / stride 1 / unpadded / undilated, or the
  // 3x3 depthwise of a MobileNetV2 block (pads 1, stride 1 or 2)
  bool conv_attrs(const Node& c, int k, int* stride, int* group) {
    if (c.as("auto_pad", "NOTSET") != "NOTSET") return false;
    const std::vector<int64_t> st = c.ais("strides"), dl = c.ais("dilations"), pd = c.ais("pads");
    for (int64_t v : dl) if (v != 1) return false;
    const int sh = st.size() > 0 ? (int)st[0] : 1, sw = st.size() > 1 ? (int)st[1] : 1;
    if (sh != sw) return false;
    for (int64_t v : pd) if (v != (k == 3 ? 1 : 0)) return false;
    if (k == 3 && pd.size() != 4) return false;
    *stride = sh;
    *group = (int)c.ai("group", 1);
    return true;
  }

  // The MobileNetV2 inverted residual starting at Conv ni — 1x1 expand ->
  // Clip -> 3x3 depthwise (stride 1 / 2) -> Clip -> 1x1 project [-> Add of
  // the block's input] — as one k_ir launch (vso_ir.hip).  1: planned (the
  // other nodes marked done), 0: not this pattern / no kernel for its shape,
  // -1: an error.
  int try_plan_ir(size_t ni) {
    if (!ir_enabled()) return 0;
    const Node& ex = g.nodes[ni];
    if (ibn.count(ni) || ex.in.size() < 2) return 0;
    // an input that is a depthwise output left to its 1x1 consumer (pending_dw:
    // no launch writes it) is computed by plan_conv's fused form, not here
    if (pending_dw.count(ex.in[0])) return 0;
    Value* x = val(ex.in[0]);
    Value* w1 = val(ex.in[1]);
    if (!x || x->is_const || x->shape.size() != 4 || !w1 || !w1->is_const || w1->c.dims.size() != 4) return 0;
    int s1, g1;
    if (!conv_attrs(ex, 1, &s1, &g1) || s1 != 1 || g1 != 1 || w1->c.dims[2] != 1 || w1->c.dims[3] != 1) return 0;
    const int N = (int)x->shape[0], CIN = (int)x->shape[1], H = (int)x->shape[2], W = (int)x->shape[3];
    const int HID = (int)w1->c.dims[0];
    if (w1->c.dims[1] != CIN) return 0;
    // the chain: each value consumed by the next node only
    const int k1 = sole_consumer(ex.out[0], ni);
    if (k1 < 0 || g.nodes[k1].op != "Clip") return 0;
    const int k2 = sole_consumer(g.nodes[k1].out[0], k1);
    if (k2 < 0 || g.nodes[k2].op != "Conv" || g.nodes[k2].in[0] != g.nodes[k1].out[0]) return 0;
    const int k3 = sole_consumer(g.nodes[k2].out[0], k2);
    if (k3 < 0 || g.nodes[k3].op != "Clip") return 0;
    const int k4 = sole_consumer(g.nodes[k3].out[0], k3);
    if (k4 < 0 || g.nodes[k4].op != "Conv" || g.nodes[k4].in[0] != g.nodes[k3].out[0]) return 0;
    const Node &dw = g.nodes[k2], &pj = g.nodes[k4];
    Value* wd = val(dw.in[1]);
    Value* w2 = val(pj.in[1]);
    int sd, gd, s2, g2;
    if (!wd || !wd->is_const || wd->c.dims.size() != 4 || !conv_attrs(dw, 3, &sd, &gd) || (sd != 1 && sd != 2) ||
        gd != HID || wd->c.dims[0] != HID || wd->c.dims[1] != 1 || wd->c.dims[2] != 3 || wd->c.dims[3] != 3)
      return 0;
    if (!w2 || !w2->is_const || w2->c.dims.size() != 4 || !conv_attrs(pj, 1, &s2, &g2) || s2 != 1 || g2 != 1 ||
        w2->c.dims[1] != HID || w2->c.dims[2] != 1 || w2->c.dims[3] != 1)
      return 0;
    const int COUT = (int)w2->c.dims[0];
    auto bias_of = [&](const Node& c, int m, std::vector<float>* b) {
      b->assign(m, 0.f);
      if (c.in.size() < 3 || c.in[2].empty()) return true;
      Value* v = val(c.in[2]);
      if (!v || !v->is_const || v->c.numel() != m) return false;
      *b = v->c.f;
      return true;
    };
    std::vector<float> b1, bd, b2;
    if (!bias_of(ex, HID, &b1) || !bias_of(dw, HID, &bd) || !bias_of(pj, COUT, &b2)) return 0;
    Epilogue c1{}, c2{};
    if (!act_of(g.nodes[k1], &c1, HID) || !act_of(g.nodes[k3], &c2, HID)) return 0;
    const int Ho = (H + 2 - 3) / sd + 1, Wo = (W + 2 - 3) / sd + 1;
    // the residual: an Add of the project's output and the block's input
    std::string out = pj.out[0];
    int k5 = sole_consumer(out, k4);
    bool res = false;
    if (k5 >= 0 && g.nodes[k5].op == "Add") {
      const Node& ad = g.nodes[k5];
      const std::string& other = ad.in[0] == out ? ad.in[1] : ad.in[0];
      if (other == ex.in[0] && ad.in[0] != ad.in[1] && sd == 1 && CIN == COUT) {
        res = true;
        out = ad.out[0];
      }
    }
    if (cat_direct.count(out) || cat_direct.count(pj.out[0])) return 0;  // (written into a Concat: the generic path)
    IrParams p{};
    p.N = N; p.CIN = CIN; p.H = H; p.W = W; p.HID = HID; p.COUT = COUT; p.Ho = Ho; p.Wo = Wo;
    p.stride = sd; p.res = res ? 1 : 0;
    p.lo1 = c1.a0; p.hi1 = c1.a1; p.lo2 = c2.a0; p.hi2 = c2.a1;
    p.b16 = s->conv_precision != PREC_F32 && ir_b16_enabled() ? 1 : 0;
    ir_tiles(Ho, Wo, &p.tiles_x, &p.tiles);
    // slices of the hidden channels: about two workgroups per CU (512; VSO_IR_WGS:
    // 256 measured 1.445 against 1.424 ms on MODNet batch 8 bf16, profiles/r05f)
    // over the tiles and slices, whole 16-channel chunks per slice (b16: whole
    // chunk pairs, and the slice's weights within the LDS budget)
    static const long wgs = [] {
      const char* e = std::getenv("VSO_IR_WGS");
      return e ? std::max(1L, std::atol(e)) : 512L;
    }();
    static const int probe = [] {
      const char* e = std::getenv("VSO_IR_PROBE");
      return e ? std::atoi(e) : 0;
    }();
    p.probe = probe;
    static const bool wave_form = [] {
      const char* e = std::getenv("VSO_IR_WAVE");
      return e && e[0] == '1';
    }();
    p.wv = p.b16 && wave_form && CIN <= 64 ? 1 : 0;
    const int nch = HID / 16;
    // b16: about 6 chunks per slice, at least 256 workgroups (VSO_IR_CPS; 0:
    // the VSO_IR_WGS target alone) — MODNet batch 8 bf16 1407.5 us of kernel
    // time against 1411 (4), 1415 (8), 1421 (the 512-workgroup target),
    // profiles/r05i
    static const int cps_target = [] {
      const char* e = std::getenv("VSO_IR_CPS");
      return e ? std::atoi(e) : 6;
    }();
    if (p.b16 && (HID % 16 != 0 || !ir_slab_plan(&p, wgs, cps_target))) return 0;
    if (!ir_supported(p)) return 0;
    if (!p.b16) {
      const long wg0 = (long)N * p.tiles;
      int ks = (int)std::min<long>(nch, std::max<long>(1, (wgs + wg0 / 2) / wg0));
      p.cps = (nch + ks - 1) / ks;
      p.ks = (nch + p.cps - 1) / p.cps;
    }
    p.pstr = ir_pstr(sd);
    // weights: the expand / project as stored ([out][in]), the depthwise tap-major
    std::vector<float> wdt((size_t)9 * HID);
    for (int h = 0; h < HID; ++h)
      for (int k = 0; k < 9; ++k) wdt[(size_t)k * HID + h] = wd->c.f[(size_t)h * 9 + k];
    flush_input(ex.in[0]);
    flush_norm(ex.in[0]);
    p.x = dptr(*x);
    p.w1 = upload_vec(w1->c.f);
    p.b1 = upload_vec(b1);
    p.wdw = upload_vec(wdt);
    p.bdw = upload_vec(bd);
    p.w2 = upload_vec(w2->c.f);
    p.b2 = upload_vec(b2);
    if (!p.w1 || !p.b1 || !p.wdw || !p.bdw || !p.w2 || !p.b2) return -1;
    if (p.b16) {
      std::vector<unsigned char> slab;
      ir_slab_build(p, w1->c.f.data(), b1.data(), wdt.data(), bd.data(), w2->c.f.data(), &slab);
      unsigned char* d = nullptr;
      if (!dalloc(&d, slab.size()) || hipMemcpy(d, slab.data(), slab.size(), hipMemcpyHostToDevice) != hipSuccess) {
        fail("constant upload failed");
        return -1;
      }
      p.slab = d;
      mark_ro(d);
    }
    if (p.ks > 1 && !dalloc(&p.part, (size_t)p.ks * N * COUT * Ho * Wo * 4)) return -1;
    if (!set_runtime(out, {N, COUT, Ho, Wo})) return -1;
    p.y = dptr(vals[out]);
    auto pp = std::make_shared<IrParams>(p);
    add(ir_kernel_name(p), [pp](hipStream_t st) { launch_ir(*pp, st); }, {reg(pp)});
    if (p.ks > 1)
      add("void vso::k_ir_reduce(vso::IrParams)", [pp](hipStream_t st) { launch_ir_reduce(*pp, st); }, {reg(pp)});
    for (int k : {k1, k2, k3, k4}) done.insert((size_t)k);
    if (res) done.insert((size_t)k5);
    s->ir_blocks++;
    return 1;
  }

  bool plan_conv(size_t ni) {
    {  // a deferred Concat copy into this Conv's input: only a dense 3x3 / 5x5
       // convolution (the k_conv_tile branch below, or its fallback, which
       // flushes) may take it; every other plan reads the whole concatenation
      const Node& cn = g.nodes[ni];
      if (cat_tail.count(cn.in[0])) {
        Value* w = cn.in.size() > 1 ? val(cn.in[1]) : nullptr;
        const bool dense = w && w->shape.size() == 4 && cn.ai("group", 1) == 1 && w->shape[2] == w->shape[3] &&
                           (w->shape[2] == 3 || w->shape[2] == 5);
        if (!dense && !flush_tail(cn.in[0])) return false;
      }
    }
    if (const int rc = try_plan_ir(ni)) return rc > 0;
    const Node& nd = g.nodes[ni];
    Value* x = val(nd.in[0]);
    Value* w = val(nd.in[1]);
    Value* b = nd.in.size() > 2 ? val(nd.in[2]) : nullptr;
    if (!w || !w->is_const) return fail("Conv '" + nd.name + "': weights must be constant");
    if (x->shape.size() != 4 || w->c.dims.size() != 4) return fail("Conv '" + nd.name + "': 2D only");
    ConvParams p{};
    p.N = (int)x->shape[0]; p.C = (int)x->shape[1]; p.H = (int)x->shape[2]; p.W = (int)x->shape[3];
    p.M = (int)w->c.dims[0]; p.Cg = (int)w->c.dims[1]; p.kh = (int)w->c.dims[2]; p.kw = (int)w->c.dims[3];
    p.G = (int)nd.ai("group", 1);
    if (p.G < 1 || p.C != p.Cg * p.G || p.M % p.G) return fail("Conv '" + nd.name + "': channel/group mismatch");
    p.Mg = p.M / p.G;
    std::vector<int64_t> st = nd.ais("strides"), dl = nd.ais("dilations"), pd = nd.ais("pads");
    p.sh = st.size() > 0 ? (int)st[0] : 1; p.sw = st.size() > 1 ? (int)st[1] : 1;
    p.dh = dl.size() > 0 ? (int)dl[0] : 1; p.dw = dl.size() > 1 ? (int)dl[1] : 1;
    int pt = pd.size() == 4 ? (int)pd[0] : 0, pl = pd.size() == 4 ? (int)pd[1] : 0;
    int pb = pd.size() == 4 ? (int)pd[2] : 0, pr = pd.size() == 4 ? (int)pd[3] : 0;
    const std::string ap = nd.as("auto_pad", "NOTSET");
    if (ap == "SAME_UPPER" || ap == "SAME_LOWER") {
      const int in[2] = {p.H, p.W}, k[2] = {p.kh, p.kw}, s2[2] = {p.sh, p.sw}, d2[2] = {p.dh, p.dw};
      int lo[2], hi[2];
      for (int d = 0; d < 2; ++d) {
        const int o = (in[d] + s2[d] - 1) / s2[d];
        const int tot = std::max((o - 1) * s2[d] + d2[d] * (k[d] - 1) + 1 - in[d], 0);
        lo[d] = ap == "SAME_UPPER" ? tot / 2 : tot - tot / 2;
        hi[d] = tot - lo[d];
      }
      pt = lo[0]; pl = lo[1]; pb = hi[0]; pr = hi[1];
    } else if (ap == "VALID") {
      pt = pl = pb = pr = 0;
    }
    p.pt = pt; p.pl = pl;
    p.Ho = (p.H + pt + pb - p.dh * (p.kh - 1) - 1) / p.sh + 1;
    p.Wo = (p.W + pl + pr - p.dw * (p.kw - 1) - 1) / p.sw + 1;
    if (p.Ho < 1 || p.Wo < 1) return fail("Conv '" + nd.name + "': empty output");
    std::vector<float> wf = w->c.f;
    std::vector<float> bias(p.M, 0.f);
    bool has_bias = false;
    if (b) {
      if (!b->is_const || b->c.numel() != p.M) return fail("Conv '" + nd.name + "': bias must be constant [M]");
      bias = b->c.f;
      has_bias = true;
    }
    // absorb BatchNormalization -> residual Add -> activation
    std::string out = nd.out[0];
    size_t last = ni;
    Epilogue ep{};
    int c1 = sole_consumer(out, last);
    const auto ib = ibn.find(ni);
    if (ib != ibn.end()) {  // an IBNorm: BN folded into channels < nb, Relu there; the InstanceNorm after the launch
      const IbnFuse& f = ib->second;
      const Node& bn = g.nodes[f.bn];
      Value *sc = val(bn.in[1]), *bb = val(bn.in[2]), *mu = val(bn.in[3]), *vr = val(bn.in[4]);
      const double eps = bn.af("epsilon", 1e-5f);
      const int64_t per = (int64_t)p.Cg * p.kh * p.kw;
      for (int m = 0; m < f.nb; ++m) {
        const double a = sc->c.f[m] / std::sqrt((double)vr->c.f[m] + eps);
        for (int64_t k = 0; k < per; ++k) wf[m * per + k] = (float)(wf[m * per + k] * a);
        bias[m] = (float)((bias[m] - mu->c.f[m]) * a + bb->c.f[m]);
      }
      has_bias = true;
      if (f.relu >= 0) {
        ep.act = ACT_RELU;
        ep.act_c_end = f.nb;
      }
      out = f.out;
      c1 = -1;
    }
    if (c1 >= 0 && g.nodes[c1].op == "BatchNormalization") {
      const Node& bn = g.nodes[c1];
      Value *sc = val(bn.in[1]), *bb = val(bn.in[2]), *mu = val(bn.in[3]), *vr = val(bn.in[4]);
      if (sc && bb && mu && vr && sc->is_const && bb->is_const && mu->is_const && vr->is_const &&
          sc->c.numel() == p.M) {
        const double eps = bn.af("epsilon", 1e-5f);
        const int64_t per = (int64_t)p.Cg * p.kh * p.kw;
        for (int m = 0; m < p.M; ++m) {
          const double a = sc->c.f[m] / std::sqrt((double)vr->c.f[m] + eps);
          for (int64_t k = 0; k < per; ++k) wf[m * per + k] = (float)(wf[m * per + k] * a);
          bias[m] = (float)((bias[m] - mu->c.f[m]) * a + bb->c.f[m]);
        }
        has_bias = true;
        done.insert((size_t)c1);
        out = bn.out[0];
        last = (size_t)c1;
        c1 = sole_consumer(out, last);
      }
    }
    const std::vector<int64_t> oshape = {p.N, p.M, p.Ho, p.Wo};
    if (c1 >= 0 && g.nodes[c1].op == "Add" && res_fuse.count(g.nodes[c1].in[0] == out ? g.nodes[c1].in[1]
                                                                                   : g.nodes[c1].in[0])) {
      const Node& ad = g.nodes[c1];
      const ResFuse& rf = res_fuse[ad.in[0] == out ? ad.in[1] : ad.in[0]];
      Value* sv = val(rf.src);
      if (!sv || sv->is_const || sv->shape.size() != 4 || sv->shape[0] != p.N || sv->shape[1] > p.M ||
          (rf.mode == 1 && (sv->shape[2] != p.Ho || sv->shape[3] != p.Wo)) ||
          (rf.mode == 2 && (sv->shape[2] / 2 != p.Ho || sv->shape[3] / 2 != p.Wo)))
        return fail("Conv '" + nd.name + "': internal: fused residual shape");
      ep.res = dptr(*sv);
      ep.res_mode = rf.mode;
      ep.res_c = (int)sv->shape[1];
      ep.res_h = (int)sv->shape[2];
      ep.res_w = (int)sv->shape[3];
      ep.out_c = p.M;
      ep.out_hw = p.Ho * p.Wo;
      ep.out_w = p.Wo;
      done.insert((size_t)c1);
      out = ad.out[0];
      last = (size_t)c1;
      c1 = sole_consumer(out, last);
    } else if (c1 >= 0 && g.nodes[c1].op == "Add") {
      const Node& ad = g.nodes[c1];
      const std::string& other = ad.in[0] == out ? ad.in[1] : ad.in[0];
      Value* o = val(other);
      if (o && !o->is_const && o->shape == oshape && ad.in[0] != ad.in[1]) {
        ep.res = dptr(*o);
        done.insert((size_t)c1);
        out = ad.out[0];
        last = (size_t)c1;
        c1 = sole_consumer(out, last);
      }
    }
    if (c1 >= 0 && is_act(g.nodes[c1].op) && act_of(g.nodes[c1], &ep, p.M)) {
      done.insert((size_t)c1);
      out = g.nodes[c1].out[0];
      last = (size_t)c1;
    }
    if (!err.empty()) return false;
    p.w = upload_vec(wf);
    ep.bias = has_bias ? upload_vec(bias) : nullptr;
    if (!p.w || (has_bias && !ep.bias)) return false;
    p.ep = ep;
    p.x = dptr(*x);
    if (!set_runtime(out, oshape)) return false;
    p.y = dptr(vals[out]);
    // (k_conv_pw stages the pair's channels in chunks: any count for a 3x3 / 5x5
    // depthwise on enough pixels; k_conv_dwpw, the rest, holds all of them in LDS)
    const int pw_m = consumer_out_channels(out, last);
    // (pw_pair_fits: pw_kernel's own test, its 32-bit offset limits included —
    // a pair it declined would fall to k_conv_dwpw, whose LDS holds kDwPwMaxC)
    const bool pw_dw = p.kh == p.kw && (p.kh == 3 || p.kh == 5) && pw_m > 0 &&
                       pw_pair_fits(p.N, p.C, (long)p.H * p.W, (long)p.Ho * p.Wo, pw_m);
    if (p.G == p.C && p.G == p.M && !ep.res && ib == ibn.end() && (pw_dw || p.C <= kDwPwMaxC) &&
        feeds_pointwise(out, last, p.M)) {
      flush_input(nd.in[0]);
      pending_dw[out] = {p.x, DwPre{p.w, p.H, p.W, p.kh, p.kw, p.sh, p.sw, p.dh, p.dw, p.pt, p.pl, ep}};
      return true;  // no launch: its 1x1 consumer computes it (k_conv_pw / k_conv_dwpw)
    }
    auto pre = pending_dw.find(nd.in[0]);
    if (pre != pending_dw.end()) {
      if (p.G != 1 || p.kh != 1 || p.kw != 1 || p.sh != 1 || p.sw != 1 || p.pt || p.pl || p.Ho != p.H || p.Wo != p.W)
        return fail("Conv '" + nd.name + "': internal: fused depthwise producer");
      p.x = pre->second.first;
      p.pre = pre->second.second;
      pending_dw.erase(pre);  // (its sole consumer: taken)
    }
    if (ib == ibn.end() && thin_conv_fits(p) && p.C <= kThinMaxC && thin_enabled()) {
      // (a matte / logit head: memory bound, on the VALU; its input's
      // InstanceNorm apply step, when left pending, folded into the loads)
      std::shared_ptr<NormParams> norm;
      auto nt = norm_pending.find(nd.in[0]);
      if (nt != norm_pending.end()) {
        norm = nt->second;
        norm_pending.erase(nt);
      }
      flush_input(nd.in[0]);  // (a pending Resize, or a Concat's pending upsampled inputs)
      auto pp = std::make_shared<ConvParams>(p);
      std::vector<Region> io{reg(pp)};
      if (norm) io.push_back(reg(norm));
      add(conv_thin_name(p.M), [pp, norm](hipStream_t st) { launch_conv_thin(*pp, norm.get(), st); }, io);
      if (cat_direct.count(out)) cat_patch[out].push_back([pp](float* base, int ctot) { retarget(pp.get(), base, ctot); });
      return true;
    }
    flush_norm(nd.in[0]);  // (a pending InstanceNorm apply step: not taken here)
    ConvTileShape ts{};
    const double macs = (double)p.N * p.M * p.Ho * p.Wo * p.Cg * p.kh * p.kw;
    const std::string* direct = cat_direct.count(out) ? &out : nullptr;
    const bool tile = !p.pre.w && conv_tile_shape(p, s->conv_precision, &ts) &&
                      (s->conv_precision != PREC_F32 || macs >= kTileMinMacs);
    // an upsampled input (or one upsampled Concat input) computed while staging
    std::vector<UpRange> ups;
    if (up_pending.count(nd.in[0])) ups.push_back({nd.in[0], 0, p.C});
    else if (cat_up.count(nd.in[0])) ups = cat_up[nd.in[0]];
    const ResizeParams* up = nullptr;
    // (one output-channel tile of at most 32 only: each tile would interpolate
    // the whole input again, and at 64 output channels the interpolation
    // measured slower than the Resize's own launch, MODNet 288x512 b8 bf16)
    static const bool up_bm64 = [] {  // (A/B knob: 64-channel upsample tiles)
      const char* e = std::getenv("VSO_UP_BM64");
      return e && e[0] == '1';
    }();
    if (tile && ups.size() == 1 && ts.s == 1 && (ts.ks == 3 || ts.ks == 5) && ts.Mp == ts.bm &&
        (ts.bm <= 32 || up_bm64) &&
        ts.prec != PREC_F32 && ups[0].c0 % 32 == 0 && ups[0].c1 % 32 == 0 && up_fuse_enabled()) {
      ConvTileShape tu{};
      tu.up = 1;
      if (conv_tile_shape(p, s->conv_precision, &tu)) {
        up = up_pending[ups[0].name].get();
        ts = tu;
      }
    }
    for (const UpRange& u : ups)
      if (!up || u.name != ups[0].name) flush_up(u.name);
    if (tile) {
      const CatTail* tail = nullptr;
      auto ct = cat_tail.find(nd.in[0]);
      if (ct != cat_tail.end() && ct->second.c0 + ct->second.C == p.C && ct->second.c0 % 32 == 0 &&
          (!up || ct->second.c0 >= ups[0].c1))
        tail = &ct->second;
      else if (!flush_tail(nd.in[0]))
        return false;
      if (!plan_conv_tile(p, ts, wf, direct, up, up ? ups[0].c0 : 0, up ? ups[0].c1 : 0, tail)) return false;
      if (tail) cat_tail.erase(nd.in[0]);
      if (up) up_pending.erase(ups[0].name);
    } else {
      if (!flush_tail(nd.in[0])) return false;
      auto pp = std::make_shared<ConvParams>(p);
      add(conv_kernel_name(p), [pp](hipStream_t st) { launch_conv(*pp, st, nullptr); }, {reg(pp)});
      if (direct) cat_patch[out].push_back([pp](float* base, int ctot) { retarget(pp.get(), base, ctot); });
    }
    if (ib != ibn.end()) {
      const IbnFuse& f = ib->second;
      const Node& inn = g.nodes[f.inorm];
      // a thin 1x1 consumer normalises its input itself: statistics only here
      const bool defer = !direct && thin_enabled() && feeds_thin(out, last);
      return plan_norm(p.y, p.y, p.N, p.M - f.nb, f.nb, p.M, (int64_t)p.Ho * p.Wo, inn, val(inn.in[1]),
                       val(inn.in[2]), f.relu >= 0 ? ACT_RELU : ACT_NONE, direct, defer ? &out : nullptr);
    }
    return true;
  }

  // `out`'s sole consumer is a Conv k_conv_thin runs (thin_conv_fits, C <= kThinMaxC)
  static constexpr int kThinMaxC = 256;
  bool feeds_thin(const std::string& out, size_t last) {
    const int c = sole_consumer(out, last);
    if (c < 0) return false;
    const Node& cv = g.nodes[c];
    if (cv.op != "Conv" || cv.in.empty() || cv.in[0] != out || cv.in.size() < 2) return false;
    Value* w = val(cv.in[1]);
    if (!w || !w->is_const || w->c.dims.size() != 4) return false;
    const std::vector<int64_t>& d = w->c.dims;
    if (d[0] > kThinMaxM || d[1] > kThinMaxC || d[2] != 1 || d[3] != 1 || cv.ai("group", 1) != 1) return false;
    for (int64_t v : cv.ais("strides")) if (v != 1) return false;
    for (int64_t v : cv.ais("pads")) if (v != 0) return false;
    const std::string ap = cv.as("auto_pad", "NOTSET");
    return ap == "NOTSET" || ap == "VALID";
  }

  static void retarget(ConvParams* p, float* base, int ctot) {
    p->y = base;
    p->y_nx = (long)(ctot - p->M) * p->Ho * p->Wo;
  }

  // A dense convolution on k_conv_tile (vso_conv.hip): weights (BatchNorm
  // folded) packed [tap][Mp][Cp] in the operand type, zero padded; a
  // partial-sum buffer when the channel chunks are split over workgroups.
  static constexpr double kTileMinMacs = 8e6;  // f32: smaller convs keep k_conv_small / k_conv_gemm
  bool plan_conv_tile(const ConvParams& p, const ConvTileShape& ts, const std::vector<float>& wf,
                      const std::string* direct, const ResizeParams* up = nullptr, int up_c0 = 0, int up_c1 = 0,
                      const CatTail* tail = nullptr) {
    const int taps = p.kh * p.kw;
    const size_t n = (size_t)taps * ts.Mp * ts.Cp;
    ConvTileParams tp{};
    tp.c = p;
    tp.Mp = ts.Mp; tp.Cp = ts.Cp; tp.tiles_x = ts.tiles_x; tp.ksplit = ts.ksplit; tp.cps = ts.cps;
    static const int qskip = [] {
      const char* e = std::getenv("VSO_CONV_QSKIP");
      return e ? std::atoi(e) : 1;
    }();
    tp.qskip = qskip;
    static const int xcd = [] {
      const char* e = std::getenv("VSO_CONV_XCD");
      return e ? std::atoi(e) : 1;
    }();
    tp.xcd = xcd;
    if (tail) {
      tp.x2 = tail->x;
      tp.x2_c0 = tail->c0;
      tp.x2_C = tail->C;
    }
    tp.tiles = ts.tiles; tp.mtiles = ts.Mp / ts.bm;
    if (up) {
      tp.up = up->x;
      tp.up_H = up->H; tp.up_W = up->W;
      tp.up_c0 = up_c0; tp.up_c1 = up_c1;
    }
    auto src = [&](size_t tap, int m, int c) { return wf[((size_t)m * p.C + c) * taps + tap]; };
    void* d = nullptr;
    if (ts.prec == PREC_F32) {
      std::vector<float> w(n, 0.f);
      for (int tap = 0; tap < taps; ++tap)
        for (int m = 0; m < p.M; ++m)
          for (int c = 0; c < p.C; ++c) w[((size_t)tap * ts.Mp + m) * ts.Cp + c] = src(tap, m, c);
      if (!dalloc(&d, n * 4) || hipMemcpy(d, w.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess)
        return fail("conv weight upload failed");
    } else {
      std::vector<uint16_t> w(n, 0);
      for (int tap = 0; tap < taps; ++tap)
        for (int m = 0; m < p.M; ++m)
          for (int c = 0; c < p.C; ++c)
            w[((size_t)tap * ts.Mp + m) * ts.Cp + c] =
                ts.prec == PREC_BF16 ? float_to_bf16(src(tap, m, c)) : float_to_half_bits(src(tap, m, c));
      if (!dalloc(&d, n * 2) || hipMemcpy(d, w.data(), n * 2, hipMemcpyHostToDevice) != hipSuccess)
        return fail("conv weight upload failed");
    }
    tp.wp = d;
    mark_ro(d);
    if (ts.ksplit > 1) {
      const size_t blocks = (size_t)p.N * (ts.Mp / ts.bm) * ts.tiles;
      // partial tiles in accumulator order: per output block and split, 256 threads x bm/16 x th*tw/64 f4
      const size_t per = (size_t)256 * (ts.bm / 16) * (ts.th * ts.tw / 64) * 16;
      if (!dalloc(&tp.part, blocks * ts.ksplit * per) || !dalloc(&tp.counters, blocks * 4))
        return false;
      if (hipMemset(tp.counters, 0, blocks * 4) != hipSuccess) return fail("hipMemset failed");
    }
    auto tpp = std::make_shared<ConvTileParams>(tp);
    add(conv_tile_name(ts), [tpp, ts](hipStream_t st) { launch_conv_tile(*tpp, ts, st); }, {reg(tpp)});
    if (direct) cat_patch[*direct].push_back([tpp](float* base, int ctot) { retarget(&tpp->c, base, ctot); });
    s->tile_convs++;
    return true;
  }

  // The output of a depthwise conv feeds exactly one Conv, 1x1 / stride 1 /
  // unpadded / ungrouped, on all its channels: the pair runs as k_conv_dwpw.
  // output channels of the sole Conv consuming `out` (its weights' dims[0]), or 0
  int consumer_out_channels(const std::string& out, size_t last) {
    const int c = sole_consumer(out, last);
    if (c < 0 || g.nodes[c].op != "Conv" || g.nodes[c].in.size() < 2) return 0;
    Value* w = val(g.nodes[c].in[1]);
    return (w && w->is_const && !w->c.dims.empty()) ? (int)w->c.dims[0] : 0;
  }

  bool feeds_pointwise(const std::string& out, size_t last, int channels) {
    const int c = sole_consumer(out, last);
    if (c < 0 || g.nodes[c].op != "Conv" || g.nodes[c].in.empty() || g.nodes[c].in[0] != out) return false;
    const Node& pw = g.nodes[c];
    Value* w = val(pw.in[1]);
    if (!w || !w->is_const || w->c.dims.size() != 4 || w->c.dims[1] != channels || w->c.dims[2] != 1 ||
        w->c.dims[3] != 1 || pw.ai("group", 1) != 1 || pw.as("auto_pad", "NOTSET") != "NOTSET")
      return false;
    for (int64_t v : pw.ais("strides")) if (v != 1) return false;
    for (int64_t v : pw.ais("pads")) if (v != 0) return false;
    for (int64_t v : pw.ais("dilations")) if (v != 1) return false;
    return true;
  }

  static void fill_strides(const std::vector<int64_t>& shape, std::vector<int64_t>* st) {
    st->assign(shape.size(), 1);
    for (int k = (int)shape.size() - 2; k >= 0; --k) (*st)[k] = (*st)[k + 1] * shape[k + 1];
  }

  bool plan_binary(const Node& nd, Value* a, Value* b, int op) {
    const size_t ra = a->shape.size(), rb = b->shape.size(), rk = std::max(ra, rb);
    if (rk > (size_t)kMaxDims) return fail(nd.op + ": rank > 6");
    std::vector<int64_t> os(rk);
    for (size_t d = 0; d < rk; ++d) {
      const int64_t da = d + ra >= rk ? a->shape[d + ra - rk] : 1, db = d + rb >= rk ? b->shape[d + rb - rk] : 1;
      if (da != db && da != 1 && db != 1) return fail(nd.op + " '" + nd.name + "': shapes do not broadcast");
      os[d] = std::max(da, db);
    }
    std::vector<int64_t> sta, stb;
    fill_strides(a->shape, &sta);
    fill_strides(b->shape, &stb);
    BinParams p{};
    p.nd = (int)rk;
    for (size_t d = 0; d < rk; ++d) {
      p.dims[d] = (int)os[d];
      const int64_t da = d + ra >= rk ? a->shape[d + ra - rk] : 1, db = d + rb >= rk ? b->shape[d + rb - rk] : 1;
      p.sa[d] = da == 1 ? 0 : sta[d + ra - rk];
      p.sb[d] = db == 1 ? 0 : stb[d + rb - rk];
    }
    p.op = op;
    p.a = operand(*a);
    p.b = operand(*b);
    if (!p.a || !p.b) return false;
    if (!set_runtime(nd.out[0], os)) return false;
    p.y = dptr(vals[nd.out[0]]);
    p.n = vals[nd.out[0]].numel();
    auto bp = std::make_shared<BinParams>(p);
    add(binary_kernel_name(*bp), [bp](hipStream_t st) { launch_binary(*bp, st); }, {reg(bp)});
    return true;
  }

  bool plan_copy_into(const float* src, const std::vector<int64_t>& src_shape, float* dst,
                      const std::vector<int64_t>& dst_shape, const std::vector<int64_t>& iter, const std::vector<int64_t>& dst_off,
                      const std::vector<int64_t>& src_start, const std::vector<int64_t>& src_step,
                      const std::vector<int64_t>& src_perm, float fill) {
    const size_t rk = iter.size();
    if (rk > (size_t)kMaxDims) return fail("copy: rank > 6");
    std::vector<int64_t> sst, dst_st;
    fill_strides(src_shape, &sst);
    fill_strides(dst_shape, &dst_st);
    CopyParams p{};
    p.nd = (int)rk;
    p.n = 1;
    long base = 0;
    for (size_t d = 0; d < rk; ++d) {
      p.size[d] = (int)iter[d];
      p.n *= iter[d];
      p.dst_stride[d] = dst_st[d];
      base += dst_off[d] * dst_st[d];
      const int64_t sd = src_perm.empty() ? (int64_t)d : src_perm[d];
      p.src_stride[d] = sst[sd];
      p.start[d] = (int)src_start[d];
      p.step[d] = (int)src_step[d];
      p.lim[d] = (int)src_shape[sd];
    }
    p.dst_base = base;
    p.src_base = 0;
    p.src = src;
    p.dst = dst;
    p.fill = fill;
    if (p.n == 0) return true;
    // a block copy (Concat / Split / Slice of whole trailing dims, no fill):
    // rows of one contiguous run in both tensors -> k_copy_rows (16-byte moves)
    bool block = src_perm.empty();
    for (size_t d = 0; block && d < rk; ++d)
      block = src_step[d] == 1 && src_start[d] >= 0 && src_start[d] + iter[d] <= src_shape[d];
    if (block) {
      int d = (int)rk - 1;
      int64_t inner = 1;
      while (d >= 0 && iter[d] == src_shape[d] && iter[d] == dst_shape[d]) inner *= iter[d--];
      if (d >= 0) inner *= iter[d--];
      bool one_outer = true;  // at most one outer dimension left (dim 0)
      for (int k = 0; k <= d && k < (int)rk; ++k)
        if (k > 0 && iter[k] != 1) one_outer = false;
      if (one_outer && d <= 0) {
        RowCopyParams q{};
        q.src = src;
        q.dst = dst;
        q.inner = inner;
        q.rows = d == 0 ? iter[0] : 1;
        q.src_row = d == 0 ? sst[0] : 0;
        q.dst_row = d == 0 ? dst_st[0] : 0;
        int64_t sb = 0;
        for (size_t k = 0; k < rk; ++k) sb += src_start[k] * sst[k];
        q.src_base = sb;
        q.dst_base = base;
        auto qp = std::make_shared<decltype(q)>(q);
        add(row_copy_name(q), [qp](hipStream_t st) { launch_copy_rows(*qp, st); }, {reg(qp)});
        return true;
      }
    }
    auto cp = std::make_shared<CopyParams>(p);
    add("vso::k_copy(vso::CopyParams)", [cp](hipStream_t st) { launch_copy(*cp, st); }, {reg(cp)});
    return true;
  }

  bool plan_node(size_t ni) {
    const Node& nd = g.nodes[ni];
    const std::string& op = nd.op;
    std::vector<Value*> in;
    bool all_const = true;
    for (const std::string& n : nd.in) {
      if (n.empty()) { in.push_back(nullptr); continue; }
      Value* v = val(n);
      if (!v) return fail("node '" + nd.name + "' (" + op + "): input '" + n + "' is not defined");
      in.push_back(v);
      all_const = all_const && v->is_const;
    }
    if (op != "Conv" && op != "Concat")
      for (const std::string& n : nd.in) flush_up(n);
    if (op == "Shape" || (all_const && !in.empty() && op != "Conv") || op == "Constant") return fold(nd, in);
    Value* x = in.empty() ? nullptr : in[0];
    const std::vector<int64_t>& xs = x->shape;
    if (op == "Conv") return plan_conv(ni);
    if (op == "Reshape" || op == "Flatten" || op == "Squeeze" || op == "Unsqueeze") {
      std::vector<int64_t> shp;
      if (!infer_view(nd, in, &shp)) return false;
      return set_runtime(nd.out[0], shp, x->buf);
    }
    if (op == "Cast" && nd.ai("to", DT_FLOAT) == DT_FLOAT16) {
      // float16 storage semantics: round to the nearest half (the values stay
      // f32 in HBM; later ops compute in f32, a superset of the f16 precision)
      UnaryParams p{};
      p.x = dptr(*x);
      p.act = ACT_F16;
      if (!set_runtime(nd.out[0], xs)) return false;
      p.y = dptr(vals[nd.out[0]]);
      p.n = vals[nd.out[0]].numel();
      auto up = std::make_shared<UnaryParams>(p);
      add("vso::k_unary(vso::UnaryParams)", [up](hipStream_t st) { launch_unary(*up, st); }, {reg(up)});
      return true;
    }
    if (op == "Identity" || op == "Dropout" || op == "Cast") {
      if (op == "Cast" && nd.ai("to", DT_FLOAT) != DT_FLOAT) return fail("Cast of a runtime tensor to a non-float type");
      return set_runtime(nd.out[0], xs, x->buf);
    }
    if (is_act(op)) {
      Epilogue ep{};
      if (op == "PRelu") return plan_binary(nd, x, in[1], BIN_PRELU);
      if (!act_of(nd, &ep, 0)) return fail(op + " '" + nd.name + "': non-constant parameters");
      UnaryParams p{};
      p.x = dptr(*x);
      p.act = ep.act; p.a0 = ep.a0; p.a1 = ep.a1;
      if (!set_runtime(nd.out[0], xs)) return false;
      p.y = dptr(vals[nd.out[0]]);
      p.n = vals[nd.out[0]].numel();
      auto up = std::make_shared<UnaryParams>(p);
      add("vso::k_unary(vso::UnaryParams)", [up](hipStream_t st) { launch_unary(*up, st); }, {reg(up)});
      return true;
    }
    if (op == "Add" || op == "Sub" || op == "Mul" || op == "Div")
      return plan_binary(nd, in[0], in[1], op == "Add" ? BIN_ADD : op == "Sub" ? BIN_SUB : op == "Mul" ? BIN_MUL : BIN_DIV);
    if (op == "MaxPool" || op == "AveragePool") {
      if (xs.size() != 4) return fail(op + ": 2D only");
      std::vector<int64_t> k = nd.ais("kernel_shape"), st = nd.ais("strides"), dl = nd.ais("dilations"), pd = nd.ais("pads");
      if (k.size() != 2) return fail(op + ": kernel_shape must be 2D");
      PoolParams p{};
      p.N = (int)xs[0]; p.C = (int)xs[1]; p.H = (int)xs[2]; p.W = (int)xs[3];
      p.kh = (int)k[0]; p.kw = (int)k[1];
      p.sh = st.size() > 0 ? (int)st[0] : 1; p.sw = st.size() > 1 ? (int)st[1] : 1;
      p.dh = dl.size() > 0 ? (int)dl[0] : 1; p.dw = dl.size() > 1 ? (int)dl[1] : 1;
      int pt = pd.size() == 4 ? (int)pd[0] : 0, pl = pd.size() == 4 ? (int)pd[1] : 0;
      int pb = pd.size() == 4 ? (int)pd[2] : 0, pr = pd.size() == 4 ? (int)pd[3] : 0;
      const std::string ap = nd.as("auto_pad", "NOTSET");
      if (ap == "SAME_UPPER" || ap == "SAME_LOWER") {
        const int inn[2] = {p.H, p.W}, kk[2] = {p.kh, p.kw}, ss[2] = {p.sh, p.sw}, dd[2] = {p.dh, p.dw};
        int lo[2], hi[2];
        for (int d = 0; d < 2; ++d) {
          const int o = (inn[d] + ss[d] - 1) / ss[d];
          const int tot = std::max((o - 1) * ss[d] + dd[d] * (kk[d] - 1) + 1 - inn[d], 0);
          lo[d] = ap == "SAME_UPPER" ? tot / 2 : tot - tot / 2;
          hi[d] = tot - lo[d];
        }
        pt = lo[0]; pl = lo[1]; pb = hi[0]; pr = hi[1];
      }
      p.pt = pt; p.pl = pl;
      const bool ceil_mode = nd.ai("ceil_mode", 0) != 0;
      auto osz = [&](int i, int p0, int p1, int kk, int ss, int dd) {
        const int num = i + p0 + p1 - dd * (kk - 1) - 1;
        int o = (ceil_mode ? (num + ss - 1) / ss : num / ss) + 1;
        if (ceil_mode && (o - 1) * ss >= i + p0) --o;
        return o;
      };
      p.Ho = osz(p.H, pt, pb, p.kh, p.sh, p.dh);
      p.Wo = osz(p.W, pl, pr, p.kw, p.sw, p.dw);
      p.max_mode = op == "MaxPool";
      p.count_include_pad = (int)nd.ai("count_include_pad", 0);
      p.x = dptr(*x);
      if (!set_runtime(nd.out[0], {xs[0], xs[1], p.Ho, p.Wo})) return false;
      p.y = dptr(vals[nd.out[0]]);
      auto pp = std::make_shared<PoolParams>(p);
      add("vso::k_pool(vso::PoolParams)", [pp](hipStream_t st) { launch_pool(*pp, st); }, {reg(pp)});
      return true;
    }
    if (op == "GlobalAveragePool") {
      RowParams p{};
      p.x = dptr(*x);
      p.rows = xs[0] * xs[1];
      p.inner = 1;
      for (size_t d = 2; d < xs.size(); ++d) p.inner *= xs[d];
      std::vector<int64_t> os = {xs[0], xs[1]};
      for (size_t d = 2; d < xs.size(); ++d) os.push_back(1);
      if (!set_runtime(nd.out[0], os)) return false;
      p.y = dptr(vals[nd.out[0]]);
      auto rp = std::make_shared<RowParams>(p);
      add(gap_kernel_name(*rp), [rp](hipStream_t st) { launch_gap(*rp, st); }, {reg(rp)});
      return true;
    }
    if (op == "InstanceNormalization") {
      if (!in[1]->is_const || !in[2]->is_const) return fail("InstanceNormalization: constant scale/B only");
      if (xs.size() < 3) return fail("InstanceNormalization: rank >= 3 only");
      int64_t inner = 1;
      for (size_t d = 2; d < xs.size(); ++d) inner *= xs[d];
      if (!set_runtime(nd.out[0], xs)) return false;
      return plan_norm(dptr(*x), dptr(vals[nd.out[0]]), (int)xs[0], (int)xs[1], 0, (int)xs[1], inner, nd, in[1], in[2],
                       ACT_NONE);
    }
    if (op == "BatchNormalization") {
      for (int k = 1; k <= 4; ++k)
        if (!in[k]->is_const) return fail("BatchNormalization: constant parameters only");
      const int C = (int)xs[1];
      std::vector<float> sc(C), sh(C);
      const double eps = nd.af("epsilon", 1e-5f);
      for (int c = 0; c < C; ++c) {
        const double a = in[1]->c.f[c] / std::sqrt((double)in[4]->c.f[c] + eps);
        sc[c] = (float)a;
        sh[c] = (float)(in[2]->c.f[c] - in[3]->c.f[c] * a);
      }
      AffineParams p{};
      p.x = dptr(*x);
      p.C = C;
      p.inner = 1;
      for (size_t d = 2; d < xs.size(); ++d) p.inner *= xs[d];
      p.scale = upload_vec(sc);
      p.shift = upload_vec(sh);
      if (!set_runtime(nd.out[0], xs)) return false;
      p.y = dptr(vals[nd.out[0]]);
      p.n = vals[nd.out[0]].numel();
      auto ap = std::make_shared<AffineParams>(p);
      add("vso::k_affine(vso::AffineParams)", [ap](hipStream_t st) { launch_affine(*ap, st); }, {reg(ap)});
      return true;
    }
    if (op == "Softmax") {
      int64_t ax = nd.ai("axis", -1);
      if (ax < 0) ax += (int64_t)xs.size();
      if (ax != (int64_t)xs.size() - 1) return fail("Softmax: last axis only");
      RowParams p{};
      p.x = dptr(*x);
      p.inner = xs.back();
      p.rows = x->numel() / std::max<int64_t>(p.inner, 1);
      if (!set_runtime(nd.out[0], xs)) return false;
      p.y = dptr(vals[nd.out[0]]);
      auto rp = std::make_shared<RowParams>(p);
      add("vso::k_softmax(vso::RowParams)", [rp](hipStream_t st) { launch_softmax(*rp, st); }, {reg(rp)});
      return true;
    }
    if (op == "Transpose") {
      std::vector<int64_t> perm = nd.ais("perm");
      const size_t rk = xs.size();
      if (perm.empty()) for (size_t k = 0; k < rk; ++k) perm.push_back((int64_t)(rk - 1 - k));
      std::vector<int64_t> os(rk);
      for (size_t k = 0; k < rk; ++k) os[k] = xs[perm[k]];
      if (!set_runtime(nd.out[0], os)) return false;
      return plan_copy_into(dptr(*x), xs, dptr(vals[nd.out[0]]), os, os, std::vector<int64_t>(rk, 0),
                            std::vector<int64_t>(rk, 0), std::vector<int64_t>(rk, 1), perm, 0.f);
    }
    if (op == "Pad") {
      const std::string mode = nd.as("mode", "constant");
      if (mode != "constant") return fail("Pad: constant mode only");
      std::vector<int64_t> pads = nd.ais("pads");
      if (in.size() > 1 && in[1]) {
        if (!in[1]->is_const) return fail("Pad: constant pads only");
        pads = in[1]->c.is_int ? in[1]->c.i : std::vector<int64_t>(in[1]->c.f.begin(), in[1]->c.f.end());
      }
      float value = nd.af("value", 0.f);
      if (in.size() > 2 && in[2]) {
        if (!in[2]->is_const) return fail("Pad: constant value only");
        if (!in[2]->c.f.empty()) value = in[2]->c.f[0];
      }
      const size_t rk = xs.size();
      std::vector<int64_t> axes;
      if (in.size() > 3 && in[3]) axes = in[3]->c.i;
      std::vector<int64_t> pb(rk, 0), pe(rk, 0);
      if (axes.empty()) {
        if (pads.size() != 2 * rk) return fail("Pad: pads length");
        for (size_t d = 0; d < rk; ++d) { pb[d] = pads[d]; pe[d] = pads[d + rk]; }
      } else {
        for (size_t k = 0; k < axes.size(); ++k) {
          const int64_t a = axes[k] < 0 ? axes[k] + (int64_t)rk : axes[k];
          pb[a] = pads[k];
          pe[a] = pads[k + axes.size()];
        }
      }
      std::vector<int64_t> os(rk), start(rk);
      for (size_t d = 0; d < rk; ++d) { os[d] = xs[d] + pb[d] + pe[d]; start[d] = -pb[d]; }
      if (!set_runtime(nd.out[0], os)) return false;
      return plan_copy_into(dptr(*x), xs, dptr(vals[nd.out[0]]), os, os, std::vector<int64_t>(rk, 0), start,
                            std::vector<int64_t>(rk, 1), {}, value);
    }
    if (op == "Concat") {
      int64_t ax = nd.ai("axis", 0);
      const size_t rk = xs.size();
      if (ax < 0) ax += (int64_t)rk;
      std::vector<int64_t> os = xs;
      os[ax] = 0;
      for (Value* v : in) os[ax] += v->shape[ax];
      if (!set_runtime(nd.out[0], os)) return false;
      int64_t off = 0;
      for (size_t q = 0; q < in.size(); ++q) {
        Value* v = in[q];
        std::vector<int64_t> doff(rk, 0);
        doff[ax] = off;
        off += v->shape[ax];
        auto direct = cat_patch.find(nd.in[q]);
        if (direct != cat_patch.end() && rk == 4 && ax == 1) {  // its producer writes it here
          for (auto& f : direct->second) f(dptr(vals[nd.out[0]]) + doff[1] * os[2] * os[3], (int)os[1]);
          if (up_pending.count(nd.in[q]))
            cat_up[nd.out[0]].push_back({nd.in[q], (int)doff[1], (int)(doff[1] + v->shape[1])});
          continue;
        }
        flush_up(nd.in[q]);
        if (q + 1 == in.size() && rk == 4 && ax == 1 && doff[1] % 32 == 0 && doff[1] > 0 && cat_tail_enabled()) {
          const int c = sole_consumer(nd.out[0], ni);
          if (c >= 0 && g.nodes[c].op == "Conv" && g.nodes[c].in[0] == nd.out[0]) {
            const float* src = operand(*v);
            if (!src) return false;
            const std::vector<int64_t> vs = v->shape;
            float* dst = dptr(vals[nd.out[0]]);
            cat_tail[nd.out[0]] = {src, (int)doff[1], (int)v->shape[1], [this, src, vs, dst, os, doff, rk]() {
                                     return plan_copy_into(src, vs, dst, os, vs, doff, std::vector<int64_t>(rk, 0),
                                                           std::vector<int64_t>(rk, 1), {}, 0.f);
                                   }};
            continue;
          }
        }
        if (!plan_copy_into(operand(*v), v->shape, dptr(vals[nd.out[0]]), os, v->shape, doff,
                            std::vector<int64_t>(rk, 0), std::vector<int64_t>(rk, 1), {}, 0.f))
          return false;
      }
      return true;
    }
    if (op == "Split") {
      int64_t ax = nd.ai("axis", 0);
      const size_t rk = xs.size();
      if (ax < 0) ax += (int64_t)rk;
      std::vector<int64_t> sp = nd.ais("split");
      if (in.size() > 1 && in[1]) sp = in[1]->c.i;
      const int64_t k = (int64_t)nd.out.size();
      if (sp.empty()) {
        const int64_t part = (xs[ax] + k - 1) / k;
        for (int64_t q = 0; q < k; ++q) sp.push_back(std::min(part, xs[ax] - q * part));
      }
      int64_t off = 0;
      for (int64_t q = 0; q < k; ++q) {
        std::vector<int64_t> os = xs;
        os[ax] = sp[q];
        if (!set_runtime(nd.out[q], os)) return false;
        std::vector<int64_t> start(rk, 0);
        start[ax] = off;
        off += sp[q];
        if (!plan_copy_into(dptr(*x), xs, dptr(vals[nd.out[q]]), os, os, std::vector<int64_t>(rk, 0), start,
                            std::vector<int64_t>(rk, 1), {}, 0.f))
          return false;
      }
      return true;
    }
    if (op == "Slice") {
      const size_t rk = xs.size();
      auto ints = [](Value* v) { return v->c.is_int ? v->c.i : std::vector<int64_t>(v->c.f.begin(), v->c.f.end()); };
      std::vector<int64_t> st, en, axes, steps;
      if (in.size() >= 3) {
        for (size_t k = 1; k < in.size(); ++k)
          if (in[k] && !in[k]->is_const) return fail("Slice: constant starts/ends/axes/steps only");
        st = ints(in[1]); en = ints(in[2]);
        if (in.size() > 3 && in[3]) axes = ints(in[3]);
        if (in.size() > 4 && in[4]) steps = ints(in[4]);
      } else {
        st = nd.ais("starts"); en = nd.ais("ends"); axes = nd.ais("axes");
      }
      if (axes.empty()) for (size_t k = 0; k < st.size(); ++k) axes.push_back((int64_t)k);
      if (steps.empty()) steps.assign(st.size(), 1);
      std::vector<int64_t> os = xs, start(rk, 0), step(rk, 1);
      for (size_t k = 0; k < st.size(); ++k) {
        const int64_t a = axes[k] < 0 ? axes[k] + (int64_t)rk : axes[k];
        const int64_t L = xs[a], s = steps[k];
        if (s == 0) return fail("Slice: zero step");
        int64_t b = st[k] < 0 ? st[k] + L : st[k], e = en[k] < 0 ? en[k] + L : en[k];
        if (s > 0) { b = std::clamp<int64_t>(b, 0, L); e = std::clamp<int64_t>(e, 0, L); os[a] = std::max<int64_t>(0, (e - b + s - 1) / s); }
        else { b = std::clamp<int64_t>(b, 0, L - 1); e = std::clamp<int64_t>(e, -1, L - 1); os[a] = std::max<int64_t>(0, (b - e - s - 1) / (-s)); }
        start[a] = b;
        step[a] = s;
      }
      if (!set_runtime(nd.out[0], os)) return false;
      return plan_copy_into(dptr(*x), xs, dptr(vals[nd.out[0]]), os, os, std::vector<int64_t>(rk, 0), start, step, {}, 0.f);
    }
    if (op == "Resize" || op == "Upsample") {
      if (xs.size() != 4) return fail(op + ": 4D only");
      std::vector<float> scales;
      std::vector<int64_t> sizes;
      if (op == "Upsample") {
        if (in.size() > 1 && in[1] && in[1]->is_const) scales = in[1]->c.f;
        else scales = nd.attrs.count("scales") ? nd.attrs.at("scales").fs : std::vector<float>{};
      } else {
        if (in.size() > 2 && in[2]) { if (!in[2]->is_const) return fail("Resize: constant scales only"); scales = in[2]->c.f; }
        if (in.size() > 3 && in[3]) { if (!in[3]->is_const) return fail("Resize: constant sizes only"); sizes = in[3]->c.i; }
      }
      ResizeParams p{};
      p.N = (int)xs[0]; p.C = (int)xs[1]; p.H = (int)xs[2]; p.W = (int)xs[3];
      if (!sizes.empty()) {
        if (sizes.size() != 4 || sizes[0] != xs[0] || sizes[1] != xs[1]) return fail("Resize: N, C must not change");
        p.Ho = (int)sizes[2]; p.Wo = (int)sizes[3];
        p.sy = (float)p.Ho / p.H; p.sx = (float)p.Wo / p.W;
      } else {
        if (scales.size() != 4 || scales[0] != 1.f || scales[1] != 1.f) return fail("Resize: scales on H, W only");
        p.sy = scales[2]; p.sx = scales[3];
        p.Ho = (int)std::floor(p.H * (double)p.sy);
        p.Wo = (int)std::floor(p.W * (double)p.sx);
      }
      const std::string mode = nd.as("mode", "nearest");
      if (mode != "nearest" && mode != "linear" && mode != "bilinear") return fail("Resize: mode " + mode);
      p.linear = mode != "nearest";
      const std::string ctm = nd.as("coordinate_transformation_mode", op == "Upsample" ? "asymmetric" : "half_pixel");
      if (ctm == "half_pixel") p.ctm = 0;
      else if (ctm == "pytorch_half_pixel") p.ctm = 1;
      else if (ctm == "align_corners") p.ctm = 2;
      else if (ctm == "asymmetric") p.ctm = 3;
      else return fail("Resize: coordinate_transformation_mode " + ctm);
      const std::string nm = nd.as("nearest_mode", "round_prefer_floor");
      p.nearest = nm == "round_prefer_floor" ? 0 : nm == "round_prefer_ceil" ? 1 : nm == "floor" ? 2 : 3;
      p.x = dptr(*x);
      if (!set_runtime(nd.out[0], {xs[0], xs[1], p.Ho, p.Wo})) return false;
      p.y = dptr(vals[nd.out[0]]);
      if ((long)p.N * p.C * p.Ho * p.Wo >= (1L << 31)) return fail("Resize: output of 2^31 elements or more");
      auto pp = std::make_shared<ResizeParams>(p);
      if (up_cand.count(nd.out[0]) && p.linear && (p.ctm == 0 || p.ctm == 1) && p.sy == 2.f && p.sx == 2.f &&
          p.Ho == 2 * p.H && p.Wo == 2 * p.W && p.C % 32 == 0 && s->conv_precision != PREC_F32)
        up_pending[nd.out[0]] = pp;  // its consumer convolution computes it (or flush_up launches it)
      else
        add(resize_kernel_name(p), [pp](hipStream_t st) { launch_resize(*pp, st); }, {reg(pp)});
      if (cat_direct.count(nd.out[0]))
        cat_patch[nd.out[0]].push_back([pp](float* base, int ctot) {
          pp->y = base;
          pp->y_nx = (long)(ctot - pp->C) * pp->Ho * pp->Wo;
        });
      return true;
    }
    if (op == "MatMul" || op == "Gemm") {
      Value* a = in[0];
      Value* b = in[1];
      GemmParams p{};
      p.alpha = 1.f;
      p.beta = 1.f;
      std::vector<int64_t> os;
      if (op == "Gemm") {
        if (a->shape.size() != 2 || b->shape.size() != 2) return fail("Gemm: 2D operands");
        const bool ta = nd.ai("transA", 0) != 0, tb = nd.ai("transB", 0) != 0;
        p.alpha = nd.af("alpha", 1.f);
        p.beta = nd.af("beta", 1.f);
        p.batch = 1;
        p.M = (int)(ta ? a->shape[1] : a->shape[0]);
        p.K = (int)(ta ? a->shape[0] : a->shape[1]);
        p.N = (int)(tb ? b->shape[0] : b->shape[1]);
        if ((tb ? b->shape[1] : b->shape[0]) != p.K) return fail("Gemm: inner dimensions differ");
        p.sam = ta ? 1 : p.K; p.sak = ta ? p.M : 1;
        p.sbk = tb ? 1 : p.N; p.sbn = tb ? p.K : 1;
        if (in.size() > 2 && in[2]) {
          Value* c = in[2];
          const std::vector<int64_t>& cs = c->shape;
          if (cs.size() == 2) { p.scm = cs[0] == 1 ? 0 : cs[1]; p.scn = cs[1] == 1 ? 0 : 1; }
          else if (cs.size() == 1) { p.scm = 0; p.scn = cs[0] == 1 ? 0 : 1; }
          else { p.scm = 0; p.scn = 0; }
          p.c = operand(*c);
        }
        os = {p.M, p.N};
      } else {
        const std::vector<int64_t>& as_ = a->shape;
        const std::vector<int64_t>& bs = b->shape;
        if (as_.size() < 2 || bs.size() < 2) return fail("MatMul: operands of rank >= 2 only");
        p.M = (int)as_[as_.size() - 2]; p.K = (int)as_.back(); p.N = (int)bs.back();
        if (bs[bs.size() - 2] != p.K) return fail("MatMul: inner dimensions differ");
        int64_t ba = 1, bb = 1;
        for (size_t d = 0; d + 2 < as_.size(); ++d) ba *= as_[d];
        for (size_t d = 0; d + 2 < bs.size(); ++d) bb *= bs[d];
        if (bb != 1 && bb != ba) return fail("MatMul: batch broadcast beyond [B] x [1] not supported");
        p.batch = (int)ba;
        p.sab = (int64_t)p.M * p.K; p.sam = p.K; p.sak = 1;
        p.sbb = bb == 1 ? 0 : (int64_t)p.K * p.N; p.sbk = p.N; p.sbn = 1;
        os = std::vector<int64_t>(as_.begin(), as_.end() - 2);
        os.push_back(p.M);
        os.push_back(p.N);
      }
      p.a = operand(*a);
      if (op == "MatMul" && b->is_const && p.sbb == 0) {
        // a constant B stored transposed ([N][K]): k contiguous for k_gemm<true>
        std::vector<float> bt((size_t)p.K * p.N);
        for (int k = 0; k < p.K; ++k)
          for (int n2 = 0; n2 < p.N; ++n2) bt[(size_t)n2 * p.K + k] = b->c.f[(size_t)k * p.N + n2];
        p.b = upload_vec(bt);
        p.sbk = 1; p.sbn = p.K;
      } else {
        p.b = operand(*b);
      }
      if (!p.a || !p.b) return false;
      // a following elementwise activation (the SE blocks' Relu / Sigmoid) in
      // the epilogue (PRelu not: its slope's axis is ambiguous on [M, N])
      std::string out = nd.out[0];
      const int c1 = gemm_act_enabled() ? sole_consumer(out, ni) : -1;
      if (c1 >= 0 && is_act(g.nodes[c1].op) && g.nodes[c1].op != "PRelu" && act_of(g.nodes[c1], &p.ep, p.N)) {
        done.insert((size_t)c1);
        out = g.nodes[c1].out[0];
      }
      if (!set_runtime(out, os)) return false;
      p.y = dptr(vals[out]);
      auto gp = std::make_shared<decltype(p)>(p);
      add(gemm_kernel_name(p), [gp](hipStream_t st) { launch_gemm(*gp, st); }, {reg(gp)});
      return true;
    }
    if (op == "MatMulNBits") return plan_matmul_nbits(nd, in);
    return fail("unsupported operator " + op + " (node '" + nd.name + "')");
  }

  // com.microsoft MatMulNBits (the q4 layers of a q4f16 export): Y = A @ W^T
  // (+ bias), W [N][K] dequantised once at create from 4-bit blocks:
  // W[n][k] = (q - zp) * scale[n][k / block_size], q the k-th nibble of row
  // n (low nibble first), zp the packed per-block zero point (default 8).
  bool plan_matmul_nbits(const Node& nd, std::vector<Value*>& in) {
    auto opt = [&](size_t k) { return in.size() > k ? in[k] : nullptr; };
    Value *a = in[0], *bq = opt(1), *sc = opt(2), *zp = opt(3), *gidx = opt(4), *bias = opt(5);
    if (!bq || !bq->is_const || !sc || !sc->is_const || (zp && !zp->is_const) || (bias && !bias->is_const))
      return fail("MatMulNBits '" + nd.name + "': B, scales, zero_points and bias must be initializers");
    if (gidx) return fail("MatMulNBits '" + nd.name + "': g_idx is not supported");
    const int64_t K = nd.ai("K", 0), N = nd.ai("N", 0), bits = nd.ai("bits", 4), bs = nd.ai("block_size", 0);
    if (bits != 4 || bs < 16 || K <= 0 || N <= 0) return fail("MatMulNBits '" + nd.name + "': 4-bit blocks only");
    const int64_t kb = (K + bs - 1) / bs, blob = bs * bits / 8, zpb = (kb * bits + 7) / 8;
    if (bq->c.numel() != N * kb * blob || sc->c.numel() != N * kb)
      return fail("MatMulNBits '" + nd.name + "': B / scales sizes do not match K, N, block_size");
    if (zp && (!zp->c.is_int || zp->c.numel() != N * zpb))
      return fail("MatMulNBits '" + nd.name + "': only packed uint8 zero points are supported");
    if (a->shape.empty() || a->shape.back() != K) return fail("MatMulNBits '" + nd.name + "': A's last dim is not K");
    std::vector<float> w((size_t)(N * K));
    for (int64_t n = 0; n < N; ++n)
      for (int64_t b = 0; b < kb; ++b) {
        const double s = sc->c.f[n * kb + b];
        const int z = zp ? (int)((zp->c.i[n * zpb + b / 2] >> ((b & 1) * 4)) & 15) : 8;
        for (int64_t j = 0; j < bs && b * bs + j < K; ++j) {
          const int q = (int)((bq->c.i[(n * kb + b) * blob + j / 2] >> ((j & 1) * 4)) & 15);
          float v = (float)((double)(q - z) * s);
          if (sc->c.f16) v = round_half(v);
          w[n * K + b * bs + j] = v;
        }
      }
    GemmParams p{};
    p.alpha = 1.f;
    p.beta = 1.f;
    p.batch = 1;
    p.K = (int)K;
    p.N = (int)N;
    p.M = (int)(a->numel() / K);
    p.sam = K; p.sak = 1;
    p.sbn = K; p.sbk = 1;  // W stored [N][K]
    p.a = operand(*a);
    p.b = upload_vec(w);
    if (bias) {
      if (bias->c.numel() != N) return fail("MatMulNBits '" + nd.name + "': bias must have N elements");
      p.c = operand(*bias);
      p.scm = 0; p.scn = 1;
    }
    if (!p.a || !p.b || (bias && !p.c)) return false;
    std::vector<int64_t> os(a->shape.begin(), a->shape.end() - 1);
    os.push_back(N);
    if (!set_runtime(nd.out[0], os)) return false;
    p.y = dptr(vals[nd.out[0]]);
    auto gp = std::make_shared<decltype(p)>(p);
    add(gemm_kernel_name(p), [gp](hipStream_t st) { launch_gemm(*gp, st); }, {reg(gp)});
    return true;
  }

  int producer(const std::string& name) const {
    for (size_t k = 0; k < g.nodes.size(); ++k)
      for (const std::string& o : g.nodes[k].out)
        if (o == name) return (int)k;
    return -1;
  }

  // InstanceNormalization (node `nd`, constant scale / B) of planes c0 .. c0+C-1
  // of an [N][ctot][inner] tensor, as k_norm_stats + k_norm_apply
  bool plan_norm(const float* x, float* y, int N, int C, int c0, int ctot, int64_t inner, const Node& nd, Value* sc,
                 Value* sh, int act, const std::string* direct = nullptr, const std::string* defer = nullptr) {
    if (sc->c.numel() != C || sh->c.numel() != C) return fail("InstanceNormalization '" + nd.name + "': scale/B size");
    NormParams p{};
    p.x = x; p.y = y;
    p.N = N; p.C = C; p.c0 = c0; p.ctot = ctot;
    p.inner = inner;
    p.scale = upload(sc->c);
    p.shift = upload(sh->c);
    p.eps = nd.af("epsilon", 1e-5f);
    p.act = act;
    p.chunk = kNormChunk;
    p.chunks = (int)((inner + kNormChunk - 1) / kNormChunk);
    if (!p.scale || !p.shift || !dalloc(&p.stats, (size_t)N * C * std::max(p.chunks, 1) * 3 * 4)) return false;
    if (inner == 0 || N * C == 0) return true;
    auto pp = std::make_shared<NormParams>(p);
    if (!defer && norm_plane_fits(inner) && norm_plane_enabled()) {
      add(norm_plane_name(inner), [pp](hipStream_t st) { launch_norm_plane(*pp, st); }, {reg(pp)});
    } else {
      add("vso::k_norm_stats(vso::NormParams)", [pp](hipStream_t st) { launch_norm_stats(*pp, st); }, {reg(pp)});
      if (defer) {  // the apply step runs in the consumer (k_conv_thin) or, failing that, flush_up
        norm_pending[*defer] = pp;
        return true;
      }
      add("vso::k_norm_apply(vso::NormParams)", [pp](hipStream_t st) { launch_norm_apply(*pp, st); }, {reg(pp)});
    }
    if (direct)  // in place on the conv's output, wherever that now lies
      cat_patch[*direct].push_back([pp](float* base, int ctot) { pp->x = pp->y = base; pp->ctot = ctot; });
    return true;
  }

  // MODNet's IBNorm (Conv2dIBNormRelu; the authors' src/models/modnet.py):
  //   c = Conv(x); Concat(BN(Slice(c, 0:nb)), InstanceNorm(Slice(c, nb:M)), axis 1) [-> Relu]
  // with every intermediate used once.  The conv writes the concatenation
  // directly: the BatchNorm folded into its first nb output channels' weights,
  // the Relu applied to those channels in its epilogue; the InstanceNorm then
  // normalises channels nb .. M-1 in place (+ Relu).  Seven launches -> three.
  struct IbnFuse {
    int nb;
    size_t bn, inorm, concat;
    int relu;  // node index or -1
    std::string out;
  };
  std::map<size_t, IbnFuse> ibn;  // conv node -> its IBNorm

  bool slice_range(const Node& nd, int64_t C, int64_t* b, int64_t* e) {
    if (nd.op != "Slice" || nd.in.size() < 3) return false;
    auto cint = [&](size_t k, std::vector<int64_t>* out) {
      if (k >= nd.in.size() || nd.in[k].empty()) return false;
      Value* v = val(nd.in[k]);
      if (!v || !v->is_const || !v->c.is_int) return false;
      *out = v->c.i;
      return true;
    };
    std::vector<int64_t> st, en, ax{0}, sp{1};
    if (!cint(1, &st) || !cint(2, &en) || st.size() != 1 || en.size() != 1) return false;
    if (nd.in.size() > 3 && !nd.in[3].empty() && !cint(3, &ax)) return false;
    if (nd.in.size() > 4 && !nd.in[4].empty() && !cint(4, &sp)) return false;
    if (ax.size() != 1 || ax[0] != 1 || sp.size() != 1 || sp[0] != 1) return false;
    *b = std::clamp<int64_t>(st[0] < 0 ? st[0] + C : st[0], 0, C);
    *e = std::clamp<int64_t>(en[0] < 0 ? en[0] + C : en[0], 0, C);
    return true;
  }

  void find_ibnorm() {
    for (size_t k = 0; k < g.nodes.size(); ++k) {
      const Node& cat = g.nodes[k];
      if (cat.op != "Concat" || cat.in.size() != 2 || cat.ai("axis", 0) != 1) continue;
      const int pbn = producer(cat.in[0]), pin = producer(cat.in[1]);
      if (pbn < 0 || pin < 0 || g.nodes[pbn].op != "BatchNormalization" || g.nodes[pin].op != "InstanceNormalization")
        continue;
      if (sole_consumer(cat.in[0], (size_t)pbn) != (int)k || sole_consumer(cat.in[1], (size_t)pin) != (int)k) continue;
      const Node &bn = g.nodes[pbn], &inn = g.nodes[pin];
      bool consts = bn.in.size() == 5 && inn.in.size() == 3;
      for (size_t q = 1; consts && q < bn.in.size(); ++q) consts = val(bn.in[q]) && val(bn.in[q])->is_const;
      for (size_t q = 1; consts && q < inn.in.size(); ++q) consts = val(inn.in[q]) && val(inn.in[q])->is_const;
      if (!consts) continue;
      const int sa = producer(bn.in[0]), sb = producer(inn.in[0]);
      if (sa < 0 || sb < 0 || sole_consumer(bn.in[0], (size_t)sa) != pbn || sole_consumer(inn.in[0], (size_t)sb) != pin)
        continue;
      const Node &la = g.nodes[sa], &lb = g.nodes[sb];
      if (la.op != "Slice" || lb.op != "Slice" || la.in[0] != lb.in[0]) continue;
      const std::string& c = la.in[0];
      const int pc = producer(c);
      if (pc < 0 || g.nodes[pc].op != "Conv" || consumers[c] != 2) continue;
      bool is_out = false;
      for (const IO& o : g.outputs) is_out = is_out || o.name == c;
      Value* wv = val(g.nodes[pc].in[1]);
      if (is_out || !wv || !wv->is_const || wv->c.dims.size() != 4) continue;
      const int64_t M = wv->c.dims[0];
      int64_t b0, e0, b1, e1;
      if (!slice_range(la, M, &b0, &e0) || !slice_range(lb, M, &b1, &e1)) continue;
      if (b0 != 0 || e0 != b1 || e1 != M || e0 <= 0 || e0 >= M) continue;
      if (val(bn.in[1])->c.numel() != e0 || val(inn.in[1])->c.numel() != M - e0) continue;
      IbnFuse f{(int)e0, (size_t)pbn, (size_t)pin, k, -1, cat.out[0]};
      const int r = sole_consumer(cat.out[0], k);
      if (r >= 0 && g.nodes[r].op == "Relu") {
        f.relu = r;
        f.out = g.nodes[r].out[0];
      }
      for (size_t q : {(size_t)sa, (size_t)sb, (size_t)pbn, (size_t)pin, k}) done.insert(q);
      if (f.relu >= 0) done.insert((size_t)f.relu);
      ibn[(size_t)pc] = f;
    }
  }

  // MaxPool(2x2, stride 2, unpadded, floor) -> [Pad: zeros appended on the
  // channel axis only] -> Add(x, Conv(...)) where the Conv's output feeds only
  // that Add (so plan_conv absorbs the Add): the Pad / MaxPool launches are
  // dropped and the conv's epilogue reads the pool input (BlazeFace's and the
  // landmark net's strided residual path: 5 + 8 launches).
  void find_residual_fusions() {
    for (size_t a = 0; a < g.nodes.size(); ++a) {
      const Node& ad = g.nodes[a];
      if (ad.op != "Add" || ad.in.size() != 2 || ad.in[0] == ad.in[1]) continue;
      for (int side = 0; side < 2; ++side) {
        const std::string& cv = ad.in[side];
        const std::string& o = ad.in[1 - side];
        const int pc = producer(cv);
        if (pc < 0 || g.nodes[pc].op != "Conv" || sole_consumer(cv, (size_t)pc) != (int)a) continue;
        int pn = producer(o);
        if (pn < 0 || sole_consumer(o, (size_t)pn) != (int)a) continue;
        int mode = 0, pad_node = -1;
        std::string cur = o;
        if (g.nodes[pn].op == "Pad" && channel_pad_only(g.nodes[pn])) {
          pad_node = pn;
          cur = g.nodes[pn].in[0];
          mode = 1;
          pn = producer(cur);
          if (pn >= 0 && sole_consumer(cur, (size_t)pn) != pad_node) pn = -1;
        }
        int pool_node = -1;
        if (pn >= 0 && g.nodes[pn].op == "MaxPool" && pool_2x2(g.nodes[pn])) {
          pool_node = pn;
          cur = g.nodes[pn].in[0];
          mode = 2;
        }
        if (mode == 0) continue;
        if (pad_node >= 0) done.insert((size_t)pad_node);
        if (pool_node >= 0) done.insert((size_t)pool_node);
        res_fuse[o] = ResFuse{cur, mode};
        break;
      }
    }
  }

  // VSO_UP_FUSE=0 keeps every Resize a launch of its own (A/B)
  static bool up_fuse_enabled() {
    static const bool on = [] {
      const char* e = std::getenv("VSO_UP_FUSE");
      return !(e && e[0] == '0');
    }();
    return on;
  }

  // VSO_NORM_PLANE=0: small InstanceNorm planes keep the stats + apply pair (A/B)
  static bool norm_plane_enabled() {
    static const bool on = [] {
      const char* e = std::getenv("VSO_NORM_PLANE");
      return !(e && e[0] == '0');
    }();
    return on;
  }

  // VSO_THIN=0: 1x1 heads of <= kThinMaxM outputs stay on the MFMA kernels (A/B)
  static bool thin_enabled() {
    static const bool on = [] {
      const char* e = std::getenv("VSO_THIN");
      return !(e && e[0] == '0');
    }();
    return on;
  }

  // launch a pending InstanceNorm apply step / fused Resize (by output name)
  // after all: its consumer cannot take it
  void flush_norm(const std::string& name) {
    auto nt = norm_pending.find(name);
    if (nt == norm_pending.end()) return;
    auto pp = nt->second;
    add("vso::k_norm_apply(vso::NormParams)", [pp](hipStream_t st) { launch_norm_apply(*pp, st); }, {reg(pp)});
    norm_pending.erase(nt);
  }
  void flush_up(const std::string& name) {
    flush_norm(name);
    auto it = up_pending.find(name);
    if (it == up_pending.end()) return;
    auto pp = it->second;
    add(resize_kernel_name(*pp), [pp](hipStream_t st) { launch_resize(*pp, st); }, {reg(pp)});
    up_pending.erase(it);
  }
  // a consumer that computes no upsample itself: its input's pending Resize and,
  // when the input is an in-place Concat, every pending upsampled input of it
  bool flush_tail(const std::string& name) {
    auto t = cat_tail.find(name);
    if (t == cat_tail.end()) return true;
    std::function<bool()> copy = std::move(t->second.copy);
    cat_tail.erase(t);
    return copy();
  }
  void flush_input(const std::string& name) {
    flush_tail(name);
    flush_up(name);
    auto cu = cat_up.find(name);
    if (cu != cat_up.end())
      for (const UpRange& u : cu->second) flush_up(u.name);
  }

  // Resizes whose output feeds one convolution's input, directly or as an
  // input of a Concat (written in place) that feeds one: planned as pending
  // (the Resize case of plan_node checks the kind: 2x linear half-pixel)
  void find_up_fusions() {
    for (size_t k = 0; k < g.nodes.size(); ++k) {
      const Node& rs = g.nodes[k];
      if (rs.op != "Resize" || done.count(k)) continue;
      const std::string& o = rs.out[0];
      const int c = sole_consumer(o, k);
      if (c < 0) continue;
      const Node& cn = g.nodes[c];
      if (cn.op == "Conv" && cn.in[0] == o) {
        up_cand.insert(o);
      } else if (cn.op == "Concat" && cat_direct.count(o) && cn.ai("axis", 0) == 1) {
        const int cc = sole_consumer(cn.out[0], (size_t)c);
        if (cc >= 0 && g.nodes[cc].op == "Conv" && g.nodes[cc].in[0] == cn.out[0]) up_cand.insert(o);
      }
    }
  }

  // Inputs of the Concats that may be written in place: used by that Concat
  // only, once, and neither a graph input / output nor a constant (whether the
  // producer can, and the Concat is on axis 1 of 4-D tensors, is decided when
  // they are planned: see cat_patch)
  void find_concat_direct() {
    std::set<std::string> fixed;
    for (const IO& o : g.inputs) fixed.insert(o.name);
    for (const IO& o : g.outputs) fixed.insert(o.name);
    for (auto& kv : g.inits) fixed.insert(kv.first);
    for (size_t k = 0; k < g.nodes.size(); ++k) {
      const Node& cat = g.nodes[k];
      if (cat.op != "Concat" || done.count(k)) continue;
      for (const std::string& i : cat.in)
        if (!i.empty() && !fixed.count(i) && consumers[i] == 1) cat_direct.insert(i);
    }
  }

  bool channel_pad_only(const Node& nd) {
    if (nd.as("mode", "constant") != "constant" || nd.in.size() < 2) return false;
    Value* pv = val(nd.in[1]);
    if (!pv || !pv->is_const || !pv->c.is_int || pv->c.i.size() != 8) return false;
    if (nd.in.size() > 2 && !nd.in[2].empty()) {
      Value* cv = val(nd.in[2]);
      if (!cv || !cv->is_const || (!cv->c.f.empty() && cv->c.f[0] != 0.f)) return false;
    }
    if (nd.in.size() > 3 && !nd.in[3].empty()) return false;  // axes
    const std::vector<int64_t>& q = pv->c.i;
    for (int d = 0; d < 8; ++d)
      if (d != 5 && q[d] != 0) return false;
    return q[5] >= 0;
  }

  static bool pool_2x2(const Node& nd) {
    const std::vector<int64_t> k = nd.ais("kernel_shape"), st = nd.ais("strides"), pd = nd.ais("pads"),
                               dl = nd.ais("dilations");
    if (k != std::vector<int64_t>{2, 2} || st != std::vector<int64_t>{2, 2}) return false;
    for (int64_t v : pd) if (v != 0) return false;
    for (int64_t v : dl) if (v != 1) return false;
    return nd.ai("ceil_mode", 0) == 0 && nd.as("auto_pad", "NOTSET") == "NOTSET";
  }

  bool run(const std::vector<std::vector<int64_t>>& in_shapes) {
    for (const Node& nd : g.nodes)
      for (const std::string& i : nd.in)
        if (!i.empty()) consumers[i]++;
    for (auto& kv : g.inits) set_const(kv.first, kv.second);
    for (size_t k = 0; k < g.inputs.size(); ++k) {
      if (!set_runtime(g.inputs[k].name, in_shapes[k])) return false;
      s->in_names.push_back(g.inputs[k].name);
      s->in_shapes.push_back(in_shapes[k]);
      s->in_bufs.push_back(vals[g.inputs[k].name].buf);
    }
    find_residual_fusions();
    find_ibnorm();
    find_concat_direct();
    if (s->conv_precision != PREC_F32) find_up_fusions();
    for (size_t k = 0; k < g.nodes.size(); ++k) {
      if (done.count(k)) continue;
      if (!plan_node(k)) return false;
    }
    if (!up_pending.empty()) return fail("internal: Resize '" + up_pending.begin()->first + "' never launched");
    if (!cat_tail.empty()) return fail("internal: Concat input copy into '" + cat_tail.begin()->first + "' never launched");
    if (!norm_pending.empty()) return fail("internal: InstanceNorm of '" + norm_pending.begin()->first + "' never applied");
    if (!pending_dw.empty()) return fail("internal: depthwise Conv into '" + pending_dw.begin()->first + "' never computed");
    for (const IO& o : g.outputs) {
      Value* v = val(o.name);
      if (!v) return fail("graph output '" + o.name + "' is never produced");
      if (v->is_const) {  // a constant output: materialise it once
        const float* d = upload(v->c);
        if (!d) return false;
        const int b = new_buf(v->c.numel());
        if (b < 0) return false;
        if (hipMemcpy(s->bufs[b], d, v->c.numel() * 4, hipMemcpyDeviceToDevice) != hipSuccess)
          return fail("constant output copy failed");
        v->buf = b;
      }
      s->out_names.push_back(o.name);
      s->out_shapes.push_back(v->shape);
      s->out_bufs.push_back(v->buf);
    }
    return true;
  }
};

int fail_s(vso_session* s, int code, const std::string& m) {
  if (s) s->err = m;
  else g_err = m;
  return code;
}

int64_t numel(const std::vector<int64_t>& v) {
  int64_t n = 1;
  for (int64_t d : v) n *= d;
  return n;
}

// Two capture lanes (VSO_LANES=1: one).  Launch i uses the device allocations
// its parameter regions point into (constants excepted); it depends on the
// last earlier launch that used each of them (every use counts as a write, so
// the users of an allocation form one chain).  List scheduling in launch
// order, unit costs: a launch starts on the lane where it can start first
// (ties: the lane of its latest dependency, then lane 0); a dependency on the
// other lane becomes an event edge.  MODNet: the HR branch's entry (the
// image resizes, e2 / e4, the first HR convolutions) runs on lane 1 beside
// the backbone's latency-bound blocks (tools/micro/graph_branches.hip:
// independent branches of one captured graph run concurrently).
struct LaneSchedule {
  std::vector<int> lane, wait_on;  // wait_on: the other lane's launch to wait for, or -1
  std::vector<char> record;        // an event is recorded after this launch
  int used = 1;
};

static LaneSchedule schedule_lanes(const vso_session* s, int lanes) {
  const size_t n = s->launches.size();
  LaneSchedule ls;
  ls.lane.assign(n, 0);
  ls.wait_on.assign(n, -1);
  ls.record.assign(n, 0);
  if (lanes < 2 || n < 2) return ls;
  std::vector<DevRange> rs = s->ranges;
  std::sort(rs.begin(), rs.end(), [](const DevRange& a, const DevRange& b) { return a.lo < b.lo; });
  auto find = [&](uintptr_t v) -> int {
    size_t lo = 0, hi = rs.size();
    while (lo < hi) {  // the last range with lo <= v
      const size_t mid = (lo + hi) / 2;
      if (rs[mid].lo <= v) lo = mid + 1;
      else hi = mid;
    }
    if (lo == 0) return -1;
    const DevRange& r = rs[lo - 1];
    return v < r.hi && !r.ro ? (int)(lo - 1) : -1;
  };
  std::vector<int> last(rs.size(), -1), fin(n, 0);
  int ready_at[2] = {0, 0};
  for (size_t i = 0; i < n; ++i) {
    std::set<int> deps;
    std::set<int> used;
    // a launch that registered no parameter block: unknown buffers, so it
    // conflicts with every buffer (ordered after and before everything)
    if (s->launches[i].io.empty())
      for (int k = 0; k < (int)rs.size(); ++k) used.insert(k);
    for (const Region& rg : s->launches[i].io)
      for (size_t o = 0; o + 8 <= rg.n; o += 8) {
        uint64_t v;
        std::memcpy(&v, static_cast<const char*>(rg.p) + o, 8);
        const int k = find((uintptr_t)v);
        if (k >= 0) used.insert(k);
      }
    for (int k : used)
      if (last[k] >= 0) deps.insert(last[k]);
    int ready = 0, latest = -1;
    for (int d : deps) {
      ready = std::max(ready, fin[d]);
      if (latest < 0 || fin[d] > fin[latest]) latest = d;
    }
    int best = 0, best_start = std::max(ready, ready_at[0]);
    const int s1 = std::max(ready, ready_at[1]);
    if (s1 < best_start || (s1 == best_start && latest >= 0 && ls.lane[latest] == 1)) {
      best = 1;
      best_start = s1;
    }
    ls.lane[i] = best;
    fin[i] = best_start + 1;
    ready_at[best] = fin[i];
    int w = -1;
    for (int d : deps)
      if (ls.lane[d] != best) w = std::max(w, d);
    if (w >= 0) {
      ls.wait_on[i] = w;
      ls.record[w] = 1;
    }
    for (int k : used) last[k] = (int)i;
    if (best == 1) ls.used = 2;
  }
  return ls;
}

// Two lanes for sessions of >= 2^21 input elements (MODNet batch 8 at
// 288x512: 1.41 -> 1.35 ms bf16, 3.88 -> 3.72 f32), one below: at batch 1 and
// on the MediaPipe nets the cross-lane edges cost more than the overlap gives
// (MODNet batch 1 0.594 -> 0.62 ms, the face detector 0.405 -> 0.447 ms;
// profiles/r05u).  VSO_LANES=1 / 2 forces either.
static int lanes_wanted(const vso_session* s) {
  static const int forced = [] {
    const char* e = std::getenv("VSO_LANES");
    return e ? std::max(1, std::min(2, std::atoi(e))) : 0;
  }();
  if (forced) return forced;
  return !s->in_shapes.empty() && numel(s->in_shapes[0]) >= (int64_t{1} << 21) ? 2 : 1;
}

int run_graph(vso_session* s, hipStream_t st) {
  if (!s->graph) {  // capture the launch list once (buffers are the session's own)
    hipGraph_t g = nullptr;
    hipStream_t cs = s->stream;
    const LaneSchedule ls = schedule_lanes(s, lanes_wanted(s));
    if (ls.used > 1 && !s->side && hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking) != hipSuccess)
      return fail_s(s, VSO_E_HIP, "hipStreamCreate failed");
    const size_t n = s->launches.size();
    std::vector<hipEvent_t> ev(n, nullptr);
    hipEvent_t fork = nullptr, join = nullptr;
    if (ls.used > 1) {
      for (size_t i = 0; i < n; ++i)
        if (ls.record[i]) {
          if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess)
            return fail_s(s, VSO_E_HIP, "hipEventCreate failed");
          s->events.push_back(ev[i]);
        }
      if (hipEventCreateWithFlags(&fork, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&join, hipEventDisableTiming) != hipSuccess)
        return fail_s(s, VSO_E_HIP, "hipEventCreate failed");
      s->events.push_back(fork);
      s->events.push_back(join);
    }
    if (hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed) != hipSuccess)
      return fail_s(s, VSO_E_HIP, "hipStreamBeginCapture failed");
    bool ok = true;
    if (ls.used > 1)  // the side lane joins the capture
      ok = hipEventRecord(fork, cs) == hipSuccess && hipStreamWaitEvent(s->side, fork, 0) == hipSuccess;
    for (size_t i = 0; i < n && ok; ++i) {
      hipStream_t ls_st = ls.lane[i] ? s->side : cs;
      if (ls.wait_on[i] >= 0) ok = hipStreamWaitEvent(ls_st, ev[ls.wait_on[i]], 0) == hipSuccess;
      if (!ok) break;  // (never captured without its cross-lane dependency)
      s->launches[i].fn(ls_st);
      if (ls.record[i]) ok = hipEventRecord(ev[i], ls_st) == hipSuccess;
    }
    if (ls.used > 1) {  // the side lane rejoins the capture, also after a failure (so it can end)
      const bool joined = hipEventRecord(join, s->side) == hipSuccess && hipStreamWaitEvent(cs, join, 0) == hipSuccess;
      ok = ok && joined;
    }
    const hipError_t e = hipStreamEndCapture(cs, &g);
    if (!ok) {
      if (g) (void)hipGraphDestroy(g);
      if (s->side) {  // whatever capture state it was left in: a fresh side stream next time
        (void)hipStreamDestroy(s->side);
        s->side = nullptr;
      }
      return fail_s(s, VSO_E_HIP, "capturing the lane schedule failed");
    }
    s->lanes_used = ls.used;
    if (e != hipSuccess || !g) return fail_s(s, VSO_E_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
    const hipError_t e2 = hipGraphInstantiate(&s->graph, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e2 != hipSuccess) return fail_s(s, VSO_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e2));
  }
  if (hipGraphLaunch(s->graph, st) != hipSuccess) return fail_s(s, VSO_E_HIP, "hipGraphLaunch failed");
  return VSO_OK;
}

struct Busy {
  vso_session* s;
  bool ok;
  explicit Busy(vso_session* ss) : s(ss) {
    int z = 0;
    ok = s->busy.compare_exchange_strong(z, 1);
  }
  ~Busy() { if (ok) s->busy.store(0); }
};

}  // namespace

extern "C" {

void vso_options_default(vso_options* o) {
  if (!o) return;
  std::memset(o, 0, sizeof *o);
  o->conv_precision = VSO_PRECISION_F32;
}

int vso_create(const void* model, size_t bytes, const int64_t* input_dims, int input_ndim, int device_id,
               vso_session** out) {
  return vso_create_ex(model, bytes, input_dims, input_ndim, device_id, nullptr, out);
}

int vso_create_ex(const void* model, size_t bytes, const int64_t* input_dims, int input_ndim, int device_id,
                  const vso_options* opts, vso_session** out) {
  if (!model || !bytes || !out) return fail_s(nullptr, VSO_E_INVALID_ARG, "null model/out");
  vso_options o;
  vso_options_default(&o);
  if (opts) o = *opts;
  if (o.conv_precision < VSO_PRECISION_F32 || o.conv_precision > VSO_PRECISION_F16)
    return fail_s(nullptr, VSO_E_INVALID_ARG, "conv_precision must be VSO_PRECISION_F32, _BF16 or _F16");
  *out = nullptr;
  Graph g;
  std::string err;
  if (!parse_model(static_cast<const uint8_t*>(model), bytes, &g, &err)) return fail_s(nullptr, VSO_E_PARSE, err);
  if (g.inputs.empty()) return fail_s(nullptr, VSO_E_UNSUPPORTED, "model has no runtime inputs");
  std::vector<std::vector<int64_t>> shapes;
  for (size_t k = 0; k < g.inputs.size(); ++k) {
    std::vector<int64_t> d = g.inputs[k].dims;
    if (k == 0 && input_dims && input_ndim > 0) d.assign(input_dims, input_dims + input_ndim);
    for (int64_t v : d)
      if (v < 1) return fail_s(nullptr, VSO_E_INVALID_ARG, "input '" + g.inputs[k].name + "' has symbolic dims: pass input_dims");
    shapes.push_back(d);
  }
  vso_session* s = new vso_session();
  s->device = device_id;
  s->conv_precision = o.conv_precision;
  if (hipSetDevice(device_id) != hipSuccess) {
    delete s;
    return fail_s(nullptr, VSO_E_HIP, "hipSetDevice failed");
  }
  if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
    delete s;
    return fail_s(nullptr, VSO_E_HIP, "hipStreamCreate failed");
  }
  Planner pl{s, g};
  if (!pl.run(shapes)) {
    const std::string m = pl.err;
    const bool unsup = m.find("unsupported") != std::string::npos || m.find("only") != std::string::npos;
    vso_destroy(s);
    return fail_s(nullptr, unsup ? VSO_E_UNSUPPORTED : VSO_E_INVALID_ARG, m);
  }
  *out = s;
  return VSO_OK;
}

void vso_destroy(vso_session* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  if (s->graph) (void)hipGraphExecDestroy(s->graph);
  for (hipEvent_t e : s->events) (void)hipEventDestroy(e);
  for (void* p : s->allocs) (void)hipFree(p);
  if (s->side) (void)hipStreamDestroy(s->side);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

const char* vso_last_error(const vso_session* s) { return s ? s->err.c_str() : g_err.c_str(); }

int vso_io_count(const vso_session* s, int* n_in, int* n_out) {
  if (!s) return VSO_E_INVALID_ARG;
  if (n_in) *n_in = (int)s->in_names.size();
  if (n_out) *n_out = (int)s->out_names.size();
  return VSO_OK;
}

static int copy_name(const std::vector<std::string>& v, int i, char* buf, int cap) {
  if (i < 0 || i >= (int)v.size() || !buf || cap < 1) return VSO_E_INVALID_ARG;
  std::snprintf(buf, (size_t)cap, "%s", v[i].c_str());
  return (int)v[i].size();
}

static int copy_shape(const std::vector<std::vector<int64_t>>& v, int i, int64_t* dims, int cap) {
  if (i < 0 || i >= (int)v.size() || !dims) return VSO_E_INVALID_ARG;
  const int n = (int)v[i].size();
  for (int k = 0; k < n && k < cap; ++k) dims[k] = v[i][k];
  return n;
}

int vso_input_name(const vso_session* s, int i, char* buf, int cap) { return s ? copy_name(s->in_names, i, buf, cap) : VSO_E_INVALID_ARG; }
int vso_output_name(const vso_session* s, int i, char* buf, int cap) { return s ? copy_name(s->out_names, i, buf, cap) : VSO_E_INVALID_ARG; }
int vso_input_shape(const vso_session* s, int i, int64_t* dims, int cap) { return s ? copy_shape(s->in_shapes, i, dims, cap) : VSO_E_INVALID_ARG; }
int vso_output_shape(const vso_session* s, int i, int64_t* dims, int cap) { return s ? copy_shape(s->out_shapes, i, dims, cap) : VSO_E_INVALID_ARG; }

int vso_run(vso_session* s, const float* const* inputs, float* const* outputs) {
  if (!s) return fail_s(nullptr, VSO_E_INVALID_ARG, "null session");
  if (!inputs || !outputs) return fail_s(s, VSO_E_INVALID_ARG, "null inputs/outputs");
  Busy b(s);
  if (!b.ok) return fail_s(s, VSO_E_INVALID_ARG, "a run is already in flight on this session");
  if (hipSetDevice(s->device) != hipSuccess) return fail_s(s, VSO_E_HIP, "hipSetDevice failed");
  for (size_t k = 0; k < s->in_bufs.size(); ++k) {
    if (!inputs[k]) return fail_s(s, VSO_E_INVALID_ARG, "null input " + std::to_string(k));
    if (hipMemcpyAsync(s->bufs[s->in_bufs[k]], inputs[k], numel(s->in_shapes[k]) * 4, hipMemcpyHostToDevice,
                       s->stream) != hipSuccess)
      return fail_s(s, VSO_E_HIP, "input copy failed");
  }
  int rc = run_graph(s, s->stream);
  if (rc) return rc;
  for (size_t k = 0; k < s->out_bufs.size(); ++k) {
    if (!outputs[k]) return fail_s(s, VSO_E_INVALID_ARG, "null output " + std::to_string(k));
    if (hipMemcpyAsync(outputs[k], s->bufs[s->out_bufs[k]], numel(s->out_shapes[k]) * 4, hipMemcpyDeviceToHost,
                       s->stream) != hipSuccess)
      return fail_s(s, VSO_E_HIP, "output copy failed");
  }
  if (hipStreamSynchronize(s->stream) != hipSuccess) return fail_s(s, VSO_E_HIP, "run failed");
  return VSO_OK;
}

int vso_run_device(vso_session* s, const float* const* d_inputs, float* const* d_outputs, void* stream) {
  if (!s) return fail_s(nullptr, VSO_E_INVALID_ARG, "null session");
  if (!d_inputs || !d_outputs) return fail_s(s, VSO_E_INVALID_ARG, "null inputs/outputs");
  Busy b(s);
  if (!b.ok) return fail_s(s, VSO_E_INVALID_ARG, "a run is already in flight on this session");
  if (hipSetDevice(s->device) != hipSuccess) return fail_s(s, VSO_E_HIP, "hipSetDevice failed");
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : s->stream;
  for (size_t k = 0; k < s->in_bufs.size(); ++k)
    if (hipMemcpyAsync(s->bufs[s->in_bufs[k]], d_inputs[k], numel(s->in_shapes[k]) * 4, hipMemcpyDeviceToDevice,
                       st) != hipSuccess)
      return fail_s(s, VSO_E_HIP, "input copy failed");
  int rc = run_graph(s, st);
  if (rc) return rc;
  for (size_t k = 0; k < s->out_bufs.size(); ++k)
    if (hipMemcpyAsync(d_outputs[k], s->bufs[s->out_bufs[k]], numel(s->out_shapes[k]) * 4, hipMemcpyDeviceToDevice,
                       st) != hipSuccess)
      return fail_s(s, VSO_E_HIP, "output copy failed");
  return VSO_OK;
}

int vso_launch_count(const vso_session* s) { return s ? (int)s->launches.size() : VSO_E_INVALID_ARG; }

int vso_tile_conv_count(const vso_session* s) { return s ? s->tile_convs : VSO_E_INVALID_ARG; }
int vso_ir_block_count(const vso_session* s) { return s ? s->ir_blocks : VSO_E_INVALID_ARG; }
int vso_lane_count(const vso_session* s) { return s ? (s->graph ? s->lanes_used : 0) : VSO_E_INVALID_ARG; }


int vso_launch_name(const vso_session* s, int k, char* buf, int cap) {
  if (!s || k < 0 || k >= (int)s->launches.size() || !buf || cap < 1) return VSO_E_INVALID_ARG;
  std::snprintf(buf, (size_t)cap, "%s", s->launches[k].name.c_str());
  return (int)s->launches[k].name.size();
}

}  // extern "C"
