// Native parser of a pickled peer update (reference
// node/node.py:138 runs pickle.loads on the serialized update the trainer
// made with pickle.dumps(local_update), node/node.py:285).
//
// The same restricted stack machine as p2pdl_amd/node/inbox.py
// `_run_pickle` / `parse_legacy_storage` / `_rebuild_tensor_v2` -- the
// reference implementation the tests hold this one to -- without the
// interpreter: only the opcodes torch emits for a state_dict (protocols
// 3-5) and for the header pickles of a legacy storage blob; globals resolve
// only to torch._utils._rebuild_tensor_v2, torch.storage._load_from_bytes,
// collections.OrderedDict and the torch.<X>Storage types; every length is
// checked against the buffer; every tensor view is checked against its
// storage (non-negative integer offset, sizes, strides; the furthest
// element inside; no zero stride over a dimension > 1; no more elements
// than the storage holds).  Anything else -- and any malformed byte --
// raises pickle.UnpicklingError.  Nothing is copied: storages come back as
// (byte offset, length) of their payload inside the message.
//
// parse_update(buffer) -> (entries, storages)
//   entries : [(key, storage index, offset, sizes tuple, strides tuple)]
//             in the update's key order
//   storages: [(storage type name, numel, payload offset, payload bytes,
//              location)]
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

PyObject* g_unpickling_error = nullptr;  // pickle.UnpicklingError

struct ParseError {
  std::string msg;
};

[[noreturn]] void fail(const std::string& m) { throw ParseError{m}; }

// Objects live in the parser's arena and refer to each other by plain
// pointers: tearing down a deep or cyclic structure a peer built (200k nested
// tuples, a list holding itself) is one flat free, never a recursion.
struct Obj;
using P = Obj*;

enum class K { None, Bool, Int, BigInt, Str, Bytes, Tuple, List, Dict, Global, Storage, Tensor };
enum class G { RebuildTensorV2, LoadFromBytes, OrderedDict, StorageType };

struct Obj {
  K kind;
  int64_t i = 0;             // Int / Bool
  std::string s;             // Str (UTF-8), BigInt (little-endian signed bytes), Global storage type name
  int64_t off = 0, len = 0;  // Bytes: a byte range of the message
  std::vector<P> items;      // Tuple / List
  std::vector<std::pair<P, P>> dict;  // Dict, insertion ordered
  bool ordered = false;      // Dict made by OrderedDict()
  G g = G::OrderedDict;      // Global
  int sidx = -1;             // Storage: index into the storage list
  // Tensor
  P storage = nullptr;
  int64_t t_off = 0;
  std::vector<int64_t> size, stride;
  explicit Obj(K k) : kind(k) {}
};

struct StorageRec {
  std::string type;
  int64_t numel, data_off, data_len;
  std::string location;
};

struct Parser {
  const uint8_t* b;   // the whole message
  int64_t n;          // its length
  std::vector<StorageRec> storages;
  std::vector<std::unique_ptr<Obj>> arena;

  P mk(K k) {
    arena.push_back(std::make_unique<Obj>(k));
    return arena.back().get();
  }
  P mk_int(int64_t v) {
    P o = mk(K::Int);
    o->i = v;
    return o;
  }

  // A byte range [pos, end) of the message is one pickle stream.
  struct Stream {
    int64_t pos, end;
  };

  static bool utf8_ok(const uint8_t* p, int64_t k) {
    int64_t i = 0;
    while (i < k) {
      const uint8_t c = p[i];
      int extra;
      uint32_t cp;
      if (c < 0x80) {
        ++i;
        continue;
      } else if ((c & 0xE0) == 0xC0) {
        extra = 1;
        cp = c & 0x1F;
      } else if ((c & 0xF0) == 0xE0) {
        extra = 2;
        cp = c & 0x0F;
      } else if ((c & 0xF8) == 0xF0) {
        extra = 3;
        cp = c & 0x07;
      } else {
        return false;
      }
      if (i + extra > k - 1) return false;  // the continuation bytes must exist
      for (int e = 1; e <= extra; ++e) {
        const uint8_t d = p[i + e];
        if ((d & 0xC0) != 0x80) return false;
        cp = (cp << 6) | (d & 0x3F);
      }
      if ((extra == 1 && cp < 0x80) || (extra == 2 && cp < 0x800) || (extra == 3 && cp < 0x10000) ||
          cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF))
        return false;
      i += extra + 1;
    }
    return true;
  }

  // bytes [p, p + k) exist; no signed overflow for any k (a peer's 8-byte
  // length may be near INT64_MAX)
  void need(const Stream& st, int64_t p, int64_t k) const {
    if (k < 0 || p < 0 || p > st.end || k > st.end - p) fail("truncated pickle");
  }
  uint64_t le(const Stream& st, int64_t p, int k) const {
    need(st, p, k);
    uint64_t v = 0;
    for (int j = 0; j < k; ++j) v |= static_cast<uint64_t>(b[p + j]) << (8 * j);
    return v;
  }
  uint8_t byte(const Stream& st, int64_t p) const {
    need(st, p, 1);
    return b[p];
  }
  P str_at(const Stream& st, int64_t p, int64_t k) {
    need(st, p, k);
    if (!utf8_ok(b + p, k)) fail("malformed peer update: UnicodeDecodeError");
    P o = mk(K::Str);
    o->s.assign(reinterpret_cast<const char*>(b + p), static_cast<size_t>(k));
    return o;
  }
  P bytes_at(const Stream& st, int64_t p, int64_t k) {
    need(st, p, k);
    P o = mk(K::Bytes);
    o->off = p;
    o->len = k;
    return o;
  }

  // which globals may resolve (the Python resolve_global callbacks)
  enum class Scope { Update, StorageBlob, NoGlobal };

  P resolve(Scope sc, const std::string& module, const std::string& name) {
    if (sc == Scope::Update) {
      P o = mk(K::Global);
      if (module == "torch._utils" && name == "_rebuild_tensor_v2") o->g = G::RebuildTensorV2;
      else if (module == "torch.storage" && name == "_load_from_bytes") o->g = G::LoadFromBytes;
      else if (module == "collections" && name == "OrderedDict") o->g = G::OrderedDict;
      else fail("refusing to load global " + module + "." + name + " from a peer update");
      return o;
    }
    if (sc == Scope::StorageBlob) {
      static const char* kTypes[] = {"FloatStorage", "DoubleStorage", "HalfStorage", "BFloat16Storage",
                                     "LongStorage", "IntStorage", "ShortStorage", "CharStorage",
                                     "ByteStorage", "BoolStorage"};
      if (module == "torch")
        for (const char* t : kTypes)
          if (name == t) {
            P o = mk(K::Global);
            o->g = G::StorageType;
            o->s = name;
            return o;
          }
      fail("unexpected global " + module + "." + name + " in a tensor storage blob");
    }
    fail("unexpected global " + module + "." + name + " in a tensor storage header");
  }

  static bool is_index(const P& x) { return x->kind == K::Int && x->i >= 0; }

  // _rebuild_tensor_v2(storage, offset, size, stride, requires_grad=False, hooks=None, metadata=None)
  P rebuild_tensor(const std::vector<P>& a) {
    if (a.size() < 4 || a.size() > 7) fail("malformed peer update: TypeError: _rebuild_tensor_v2 arguments");
    const P& storage = a[0];
    const P& offset = a[1];
    const P& size = a[2];
    const P& stride = a[3];
    if (storage->kind != K::Storage) fail("tensor without a storage");
    if (size->kind != K::Tuple || stride->kind != K::Tuple || size->items.size() != stride->items.size())
      fail("tensor size / stride must be tuples of the same length");
    bool ok = is_index(offset);
    for (const P& x : size->items) ok = ok && is_index(x);
    for (const P& x : stride->items) ok = ok && is_index(x);
    if (!ok) fail("tensor offset, sizes and strides must be non-negative integers");
    const int64_t snumel = storages[storage->sidx].numel;
    const size_t d = size->items.size();
    bool nonempty = true;
    for (const P& x : size->items) nonempty = nonempty && x->i != 0;
    if (nonempty) {
      // the furthest element must exist (Python ints do not overflow: saturate)
      __int128 last = offset->i;  // every term >= 0: stop once past the storage (no overflow)
      for (size_t j = 0; j < d && last < snumel; ++j)
        last += static_cast<__int128>(size->items[j]->i - 1) * stride->items[j]->i;
      if (last >= snumel)
        fail("tensor view ends at element " + std::to_string(static_cast<long long>(
                 last > INT64_MAX ? INT64_MAX : static_cast<int64_t>(last))) +
             ", storage holds " + std::to_string(snumel));
      for (size_t j = 0; j < d; ++j)
        if (stride->items[j]->i == 0 && size->items[j]->i > 1) fail("tensor view with a zero stride");
      __int128 numel = 1;
      for (size_t j = 0; j < d; ++j) {
        numel *= size->items[j]->i;
        if (numel > snumel) break;
      }
      if (numel > snumel - offset->i)
        fail("tensor view of " + std::to_string(static_cast<long long>(numel)) + " elements over " +
             std::to_string(snumel - offset->i));
    } else if (offset->i > snumel) {
      fail("tensor offset past the end of its storage");
    }
    P t = mk(K::Tensor);
    t->storage = storage;
    t->t_off = offset->i;
    for (size_t j = 0; j < d; ++j) {
      t->size.push_back(size->items[j]->i);
      t->stride.push_back(stride->items[j]->i);
    }
    return t;
  }

  // torch legacy storage blob (torch/serialization.py _legacy_save), as
  // inbox.py parse_legacy_storage: magic, protocol version and sys_info
  // pickles, the storage record (persistent id), the key list, an int64
  // count and the raw little-endian payload.
  P load_from_bytes(const std::vector<P>& a) {
    if (a.size() != 1) fail("malformed peer update: TypeError: _load_from_bytes arguments");
    if (a[0]->kind != K::Bytes) fail("storage blob must be bytes");
    Stream st{a[0]->off, a[0]->off + a[0]->len};
    int64_t pos = st.pos;
    P magic = run(st, pos, 2, Scope::NoGlobal, nullptr);
    static const uint8_t kMagic[] = {0x6C, 0xFC, 0x9C, 0x46, 0xF9, 0x20, 0x6A, 0xA8, 0x50, 0x19};  // 0x1950A86A20F9469CFC6C
    bool magic_ok = false;
    if (magic->kind == K::BigInt) {
      // minimal two's complement little-endian: the 10 bytes, maybe a 0 pad
      const std::string& v = magic->s;
      std::string want(reinterpret_cast<const char*>(kMagic), sizeof(kMagic));
      std::string trimmed = v;
      while (trimmed.size() > 1 && trimmed.back() == '\0' && !(trimmed[trimmed.size() - 2] & 0x80)) trimmed.pop_back();
      magic_ok = trimmed == want;
    }
    if (!magic_ok) fail("not a torch legacy storage blob (magic)");
    P ver = run(st, pos, 2, Scope::NoGlobal, nullptr);
    if (ver->kind != K::Int || ver->i != 1001) fail("unsupported legacy protocol version");
    P info = run(st, pos, 2, Scope::NoGlobal, nullptr);
    bool le_ok = false;
    if (info->kind == K::Dict)
      for (auto& kv : info->dict)
        if (kv.first->kind == K::Str && kv.first->s == "little_endian")
          le_ok = kv.second->kind == K::Bool && kv.second->i == 1;
    if (!le_ok) fail("storage blob is not little-endian");
    std::vector<P> pids;
    run(st, pos, 2, Scope::StorageBlob, &pids);
    if (pids.size() != 1 || pids[0]->kind != K::Tuple || pids[0]->items.size() < 5 || pids[0]->items[0]->kind != K::Str ||
        pids[0]->items[0]->s != "storage")
      fail("storage blob without exactly one storage record");
    const auto& pid = pids[0]->items;
    const P& stype = pid[1];
    const P& key = pid[2];
    const P& location = pid[3];
    const P& numel = pid[4];
    if (stype->kind != K::Global || stype->g != G::StorageType || numel->kind != K::Int || numel->i < 0 ||
        key->kind != K::Str)
      fail("malformed storage record");
    if (pid.size() > 5 && pid[5]->kind != K::None) fail("storage views are not supported");
    if (location->kind != K::Str) fail("malformed storage record (location)");
    P keys = run(st, pos, 2, Scope::NoGlobal, nullptr);
    if (keys->kind != K::List || keys->items.size() != 1 || keys->items[0]->kind != K::Str ||
        keys->items[0]->s != key->s)
      fail("expected exactly one storage per blob");
    int item = 0;
    const std::string& t = stype->s;
    if (t == "FloatStorage" || t == "IntStorage") item = 4;
    else if (t == "DoubleStorage" || t == "LongStorage") item = 8;
    else if (t == "HalfStorage" || t == "BFloat16Storage" || t == "ShortStorage") item = 2;
    else if (t == "CharStorage" || t == "ByteStorage" || t == "BoolStorage") item = 1;
    else fail(t + " is not supported");
    if (pos + 8 > st.end) fail("truncated storage blob");
    const int64_t count = static_cast<int64_t>(le(st, pos, 8));
    const __int128 nbytes = static_cast<__int128>(count) * item;
    if (count != numel->i || pos + 8 + nbytes != st.end) fail("storage payload size mismatch");
    P s = mk(K::Storage);
    s->sidx = static_cast<int>(storages.size());
    storages.push_back(StorageRec{t, numel->i, pos + 8, static_cast<int64_t>(nbytes), location->s});
    return s;
  }

  static bool key_eq(const P& a, const P& b) {
    auto num = [](const P& x) { return x->kind == K::Int || x->kind == K::Bool; };
    if (num(a) && num(b)) return a->i == b->i;
    if (a->kind != b->kind) return false;
    switch (a->kind) {
      case K::None: return true;
      case K::Str: return a->s == b->s;
      default: return a == b;
    }
  }
  static void dict_set(P d, P k, P v) {
    if (d->kind != K::Dict) fail("malformed peer update: TypeError: SETITEM on something that is not a dict");
    if (!(k->kind == K::Str || k->kind == K::Int || k->kind == K::Bool || k->kind == K::None))
      fail("malformed peer update: unsupported dict key");
    for (auto& kv : d->dict)
      if (key_eq(kv.first, k)) {
        kv.second = v;
        return;
      }
    d->dict.emplace_back(k, v);
  }

  // One pickle of the stream from pos up to its STOP (inbox.py _run_pickle).
  P run(const Stream& st, int64_t& pos, int min_proto, Scope sc, std::vector<P>* pids) {
    std::vector<P> stack;
    std::vector<size_t> marks;
    std::unordered_map<uint64_t, P> memo;
    auto top = [&]() -> P& {  // a MARK on top is not an object here (stricter than the Python machine)
      if (stack.empty() || (!marks.empty() && marks.back() == stack.size()))
        fail("malformed peer update: IndexError: stack underflow");
      return stack.back();
    };
    auto pop = [&]() -> P {
      if (stack.empty() || (!marks.empty() && marks.back() == stack.size()))
        fail("malformed peer update: IndexError: stack underflow");
      P v = stack.back();
      stack.pop_back();
      return v;
    };
    auto pop_mark = [&]() -> std::vector<P> {
      if (marks.empty()) fail("MARK not found");
      const size_t m = marks.back();
      marks.pop_back();
      std::vector<P> items(stack.begin() + static_cast<std::ptrdiff_t>(m), stack.end());
      stack.resize(m);
      return items;
    };
    auto memo_get = [&](uint64_t idx) -> P {
      auto it = memo.find(idx);
      if (it == memo.end()) fail("malformed peer update: KeyError: memo");
      return it->second;
    };
    while (pos < st.end) {
      const uint8_t op = b[pos++];
      switch (op) {
        case 0x94:  // MEMOIZE
          memo[memo.size()] = top();
          break;
        case 0x4B:  // BININT1
          stack.push_back(mk_int(byte(st, pos)));
          pos += 1;
          break;
        case 0x71:  // BINPUT
          memo[byte(st, pos)] = top();
          pos += 1;
          break;
        case 0x58: {  // BINUNICODE
          const int64_t k = static_cast<int64_t>(le(st, pos, 4));
          stack.push_back(str_at(st, pos + 4, k));
          pos += 4 + k;
          break;
        }
        case 0x8C: {  // SHORT_BINUNICODE
          const int64_t k = byte(st, pos);
          stack.push_back(str_at(st, pos + 1, k));
          pos += 1 + k;
          break;
        }
        case 0x52: {  // REDUCE
          P args = pop();
          P fn = top();
          if (fn->kind != K::Global || fn->g == G::StorageType || args->kind != K::Tuple)
            fail("REDUCE of something that is not an allowed global");
          P r;
          if (fn->g == G::OrderedDict) {
            if (!args->items.empty()) fail("OrderedDict with arguments");
            r = mk(K::Dict);
            r->ordered = true;
          } else if (fn->g == G::LoadFromBytes) {
            r = load_from_bytes(args->items);
          } else {
            r = rebuild_tensor(args->items);
          }
          stack.back() = r;
          break;
        }
        case 0x28:  // MARK
          marks.push_back(stack.size());
          break;
        case 0x68:  // BINGET
          stack.push_back(memo_get(byte(st, pos)));
          pos += 1;
          break;
        case 0x85: {  // TUPLE1
          P t = mk(K::Tuple);
          t->items.push_back(pop());
          stack.push_back(t);
          break;
        }
        case 0x74: {  // TUPLE
          P t = mk(K::Tuple);
          t->items = pop_mark();
          stack.push_back(t);
          break;
        }
        case 0x42: {  // BINBYTES
          const int64_t k = static_cast<int64_t>(le(st, pos, 4));
          stack.push_back(bytes_at(st, pos + 4, k));
          pos += 4 + k;
          break;
        }
        case 0x89: {  // NEWFALSE
          P o = mk(K::Bool);
          o->i = 0;
          stack.push_back(o);
          break;
        }
        case 0x29:  // EMPTY_TUPLE
          stack.push_back(mk(K::Tuple));
          break;
        case 0x2E:  // STOP
          return pop();
        case 0x80:  // PROTO
          if (byte(st, pos) < min_proto)
            fail("pickle protocol " + std::to_string(b[pos]) + " (< " + std::to_string(min_proto) +
                 ") is not accepted");
          pos += 1;
          break;
        case 0x95:  // FRAME
          need(st, pos, 8);
          pos += 8;
          break;
        case 0x7D:  // EMPTY_DICT
          stack.push_back(mk(K::Dict));
          break;
        case 0x5D:  // EMPTY_LIST
          stack.push_back(mk(K::List));
          break;
        case 0x72:  // LONG_BINPUT
          memo[le(st, pos, 4)] = top();
          pos += 4;
          break;
        case 0x6A:  // LONG_BINGET
          stack.push_back(memo_get(le(st, pos, 4)));
          pos += 4;
          break;
        case 0x43: {  // SHORT_BINBYTES
          const int64_t k = byte(st, pos);
          stack.push_back(bytes_at(st, pos + 1, k));
          pos += 1 + k;
          break;
        }
        case 0x8E: {  // BINBYTES8
          const uint64_t k = le(st, pos, 8);
          if (k > static_cast<uint64_t>(st.end - (pos + 8))) fail("truncated pickle");  // before any use of k
          stack.push_back(bytes_at(st, pos + 8, static_cast<int64_t>(k)));
          pos += 8 + static_cast<int64_t>(k);
          break;
        }
        case 0x4D:  // BININT2
          stack.push_back(mk_int(static_cast<int64_t>(le(st, pos, 2))));
          pos += 2;
          break;
        case 0x4A:  // BININT (signed)
          stack.push_back(mk_int(static_cast<int32_t>(static_cast<uint32_t>(le(st, pos, 4)))));
          pos += 4;
          break;
        case 0x8A: {  // LONG1
          const int k = byte(st, pos);
          need(st, pos + 1, k);
          if (k <= 8) {
            uint64_t v = 0;
            for (int j = 0; j < k; ++j) v |= static_cast<uint64_t>(b[pos + 1 + j]) << (8 * j);
            if (k > 0 && k < 8 && (b[pos + k] & 0x80)) v |= ~uint64_t(0) << (8 * k);  // sign-extend
            stack.push_back(mk_int(static_cast<int64_t>(v)));
          } else {
            P o = mk(K::BigInt);
            o->s.assign(reinterpret_cast<const char*>(b + pos + 1), static_cast<size_t>(k));
            stack.push_back(o);
          }
          pos += 1 + k;
          break;
        }
        case 0x88: {  // NEWTRUE
          P o = mk(K::Bool);
          o->i = 1;
          stack.push_back(o);
          break;
        }
        case 0x4E:  // NONE
          stack.push_back(mk(K::None));
          break;
        case 0x86: {  // TUPLE2
          P t = mk(K::Tuple);
          P y = pop();
          P x = pop();
          t->items = {x, y};
          stack.push_back(t);
          break;
        }
        case 0x87: {  // TUPLE3
          P t = mk(K::Tuple);
          P z = pop();
          P y = pop();
          P x = pop();
          t->items = {x, y, z};
          stack.push_back(t);
          break;
        }
        case 0x93: {  // STACK_GLOBAL
          P name = pop();
          P module = pop();
          if (name->kind != K::Str || module->kind != K::Str) fail("STACK_GLOBAL needs two strings");
          stack.push_back(resolve(sc, module->s, name->s));
          break;
        }
        case 0x63: {  // GLOBAL (text: module\nname\n, each within 256 bytes)
          auto line = [&](int64_t p) -> int64_t {
            const int64_t lim = std::min<int64_t>(p + 256, st.end);
            for (int64_t q = p; q < lim; ++q)
              if (b[q] == '\n') return q;
            fail("malformed peer update: ValueError: GLOBAL without a newline");
          };
          const int64_t e1 = line(pos);
          const int64_t e2 = line(e1 + 1);
          auto ascii = [&](int64_t p, int64_t q) {
            std::string s;
            for (int64_t j = p; j < q; ++j) {
              if (b[j] >= 0x80) fail("malformed peer update: UnicodeDecodeError");
              s.push_back(static_cast<char>(b[j]));
            }
            return s;
          };
          const std::string module = ascii(pos, e1), name = ascii(e1 + 1, e2);
          pos = e2 + 1;
          stack.push_back(resolve(sc, module, name));
          break;
        }
        case 0x51: {  // BINPERSID
          if (pids == nullptr) fail("persistent ids are not accepted here");
          P pid = pop();
          pids->push_back(pid);
          stack.push_back(mk(K::None));
          break;
        }
        case 0x62: {  // BUILD: only torch's OrderedDict `_metadata`
          P state = pop();
          P inst = top();
          if (state->kind == K::Dict && inst->kind == K::Dict && inst->ordered) {
            for (auto& kv : state->dict)
              if (!(kv.first->kind == K::Str && kv.first->s == "_metadata"))
                fail("unexpected attributes on a state_dict");
          } else if (state->kind != K::None) {
            fail("unexpected BUILD");
          }
          break;
        }
        case 0x73: {  // SETITEM
          P v = pop();
          P k = pop();
          dict_set(top(), k, v);
          break;
        }
        case 0x75: {  // SETITEMS
          std::vector<P> items = pop_mark();
          P d = top();
          if (items.size() % 2) fail("malformed peer update: IndexError: odd SETITEMS");
          for (size_t j = 0; j < items.size(); j += 2) dict_set(d, items[j], items[j + 1]);
          break;
        }
        case 0x61: {  // APPEND
          P v = pop();
          P l = top();
          if (l->kind != K::List) fail("malformed peer update: AttributeError: APPEND to a non-list");
          l->items.push_back(v);
          break;
        }
        case 0x65: {  // APPENDS
          std::vector<P> items = pop_mark();
          P l = top();
          if (l->kind != K::List) fail("malformed peer update: AttributeError: APPENDS to a non-list");
          l->items.insert(l->items.end(), items.begin(), items.end());
          break;
        }
        default: {
          char buf[64];
          snprintf(buf, sizeof buf, "opcode 0x%02x is not accepted in a peer update", op);
          fail(buf);
        }
      }
    }
    fail("truncated pickle");
  }
};

PyObject* to_py_key(const P& k) {
  switch (k->kind) {
    case K::Str: return PyUnicode_DecodeUTF8(k->s.data(), static_cast<Py_ssize_t>(k->s.size()), "strict");
    case K::Int: return PyLong_FromLongLong(k->i);
    case K::Bool: return PyBool_FromLong(k->i);
    default: Py_RETURN_NONE;
  }
}

PyObject* tuple_of(const std::vector<int64_t>& v) {
  PyObject* t = PyTuple_New(static_cast<Py_ssize_t>(v.size()));
  if (!t) return nullptr;
  for (size_t j = 0; j < v.size(); ++j) {
    PyObject* x = PyLong_FromLongLong(v[j]);
    if (!x) {
      Py_DECREF(t);
      return nullptr;
    }
    PyTuple_SET_ITEM(t, static_cast<Py_ssize_t>(j), x);
  }
  return t;
}

// The whole parse, without the GIL (no Python object is touched): the
// update's (key, tensor) entries, or the error message.
std::string run_update(Parser& ps, std::vector<std::pair<P, P>>& entries) noexcept {
  try {
    int64_t pos = 0;
    P obj = ps.run(Parser::Stream{0, ps.n}, pos, 3, Parser::Scope::Update, nullptr);
    if (obj->kind != K::Dict) return "a peer update must be a dict of tensors";
    for (auto& kv : obj->dict)
      if (kv.second->kind != K::Tensor) return "a peer update must be a dict of tensors";
    entries = obj->dict;
    return {};
  } catch (ParseError& e) {
    return e.msg.empty() ? std::string("malformed peer update") : e.msg;
  } catch (std::bad_alloc&) {
    return "malformed peer update: MemoryError";
  } catch (...) {
    return "malformed peer update";
  }
}

PyObject* parse_update(PyObject*, PyObject* arg) {
  Py_buffer view;
  if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) != 0) return nullptr;
  Parser ps{static_cast<const uint8_t*>(view.buf), static_cast<int64_t>(view.len), {}, {}};
  std::vector<std::pair<P, P>> entries;
  std::string err;
  Py_BEGIN_ALLOW_THREADS
  err = run_update(ps, entries);
  Py_END_ALLOW_THREADS
  PyBuffer_Release(&view);
  if (!err.empty()) {
    PyErr_SetString(g_unpickling_error, err.c_str());
    return nullptr;
  }
  PyObject* out_e = PyList_New(static_cast<Py_ssize_t>(entries.size()));
  PyObject* out_s = PyList_New(static_cast<Py_ssize_t>(ps.storages.size()));
  if (!out_e || !out_s) {
    Py_XDECREF(out_e);
    Py_XDECREF(out_s);
    return nullptr;
  }
  for (size_t j = 0; j < entries.size(); ++j) {
    const P& t = entries[j].second;
    PyObject* key = to_py_key(entries[j].first);
    PyObject* size = key ? tuple_of(t->size) : nullptr;
    PyObject* stride = size ? tuple_of(t->stride) : nullptr;
    PyObject* item = stride ? Py_BuildValue("(NiLNN)", key, t->storage->sidx, static_cast<long long>(t->t_off),
                                            size, stride)
                            : nullptr;
    if (!item) {
      if (!stride) {
        Py_XDECREF(key);
        Py_XDECREF(size);
      }
      Py_DECREF(out_e);
      Py_DECREF(out_s);
      return nullptr;
    }
    PyList_SET_ITEM(out_e, static_cast<Py_ssize_t>(j), item);
  }
  for (size_t j = 0; j < ps.storages.size(); ++j) {
    const StorageRec& r = ps.storages[j];
    PyObject* item = Py_BuildValue("(s#LLLN)", r.type.data(), static_cast<Py_ssize_t>(r.type.size()),
                                   static_cast<long long>(r.numel), static_cast<long long>(r.data_off),
                                   static_cast<long long>(r.data_len),
                                   PyUnicode_DecodeUTF8(r.location.data(), static_cast<Py_ssize_t>(r.location.size()),
                                                        "strict"));
    if (!item) {
      Py_DECREF(out_e);
      Py_DECREF(out_s);
      return nullptr;
    }
    PyList_SET_ITEM(out_s, static_cast<Py_ssize_t>(j), item);
  }
  return Py_BuildValue("(NN)", out_e, out_s);
}

PyMethodDef methods[] = {
    {"parse_update", parse_update, METH_O,
     "parse_update(buffer) -> (entries, storages): the restricted parse of a pickled peer update"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_wire", nullptr, -1, methods, nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__wire(void) {
  PyObject* pickle = PyImport_ImportModule("pickle");
  if (!pickle) return nullptr;
  g_unpickling_error = PyObject_GetAttrString(pickle, "UnpicklingError");
  Py_DECREF(pickle);
  if (!g_unpickling_error) return nullptr;
  return PyModule_Create(&module);
}
