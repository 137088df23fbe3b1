// MessageCodec: schema-driven native protobuf codec for flat messages.
//
// Hot path of both reference handlers: `proto.decode(type, content)`
// (index.js:63, :129). The field table comes from the runtime descriptor
// built from beholder_amd/models/proto/*.proto (see ops/__init__.py), so the
// codec follows the .proto file instead of hard-coding field numbers.
// Decoded messages are PyStructSequence instances: attribute access by proto
// field name (msg.mediaId, msg.status, ...) like protobufjs / upb messages.
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "pbjs.hpp"
#include "py_common.hpp"
#include "wire.hpp"

namespace beholder {

namespace {

constexpr int MAX_FIELDS = 64;
constexpr uint32_t MAX_FIELD_NUMBER = 65535;

struct FieldSpec {
  uint32_t number;
  int kind;
};

// Decode dialects: how malformed input is read (valid input decodes the same either way).
enum Dialect : int {
  D_UPB = 0,         // google.protobuf acceptance rules (wire.hpp), the tooling / test oracle
  D_PROTOBUFJS = 1,  // protobufjs 6.8.8 BufferReader (pbjs.hpp), what the reference runs
};

struct CodecObject {
  PyObject_HEAD PyTypeObject* result_type;
  int dialect;
  bool fast_new;  // result_type has n fields, all visible: results are made by new_result()
  std::vector<int16_t>* by_number;  // field number -> slot (-1 = unknown)
  std::vector<FieldSpec>* fields;   // by slot
  PyObject* defaults;               // tuple, per slot
  PyObject* names;                  // tuple of str, per slot
  PyObject* type_name;              // str
};

// CPython 3.10's PyStructSequence_New and the struct sequence dealloc look up the type's
// `n_fields` / `n_sequence_fields` in its dict (by _Py_IDENTIFIER) on every call: three dict
// lookups per decoded message, each a hash probe of an identifier string. Our result types have
// every field visible, so the sizes are the type's item count: new_result() makes the object the
// way PyStructSequence_New does (same layout, same untracked state) without the lookups, and the
// type's dealloc is replaced by one that reads the size from the object.
static Py_ssize_t type_size_attr(PyTypeObject* t, const char* name) {
  PyObject* v = PyDict_GetItemString(t->tp_dict, name);  // borrowed
  return v && PyLong_Check(v) ? PyLong_AsSsize_t(v) : -1;
}

static void result_dealloc(PyObject* obj) {
  PyTypeObject* tp = Py_TYPE(obj);
  PyObject_GC_UnTrack(obj);
  PyTupleObject* t = reinterpret_cast<PyTupleObject*>(obj);
  for (Py_ssize_t i = 0, n = Py_SIZE(obj); i < n; ++i) Py_XDECREF(t->ob_item[i]);
  PyObject_GC_Del(obj);
  if (tp->tp_flags & Py_TPFLAGS_HEAPTYPE) Py_DECREF(tp);
}

static inline PyObject* new_result(CodecObject* self, Py_ssize_t n) {
  if (!self->fast_new) return PyStructSequence_New(self->result_type);
  PyTupleObject* obj = PyObject_GC_NewVar(PyTupleObject, self->result_type, n);
  if (!obj) return nullptr;
  for (Py_ssize_t i = 0; i < n; ++i) obj->ob_item[i] = nullptr;
  return reinterpret_cast<PyObject*>(obj);
}

union SlotVal {
  uint64_t u;
  double d;
  struct {
    const uint8_t* p;
    size_t n;
  } s;
};

PyObject* default_for(int kind) {
  switch (kind) {
    case wire::K_STRING:
      return PyUnicode_FromStringAndSize("", 0);
    case wire::K_BYTES:
      return PyBytes_FromStringAndSize("", 0);
    case wire::K_BOOL:
      Py_RETURN_FALSE;
    case wire::K_FLOAT:
    case wire::K_DOUBLE:
      return PyFloat_FromDouble(0.0);
    default:
      return PyLong_FromLong(0);
  }
}

void codec_dealloc(CodecObject* self) {
  Py_XDECREF(self->result_type);
  Py_XDECREF(self->defaults);
  Py_XDECREF(self->names);
  Py_XDECREF(self->type_name);
  delete self->by_number;
  delete self->fields;
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

PyObject* codec_new(PyTypeObject* type, PyObject*, PyObject*) {
  CodecObject* self = reinterpret_cast<CodecObject*>(type->tp_alloc(type, 0));
  if (!self) return nullptr;
  self->result_type = nullptr;
  self->fast_new = false;
  self->dialect = D_UPB;
  self->by_number = nullptr;
  self->fields = nullptr;
  self->defaults = nullptr;
  self->names = nullptr;
  self->type_name = nullptr;
  return reinterpret_cast<PyObject*>(self);
}

// MessageCodec(type_name: str, fields: sequence of (number, name, kind), dialect="upb")
int codec_init_impl(CodecObject* self, PyObject* args, PyObject* kwds);
int codec_init(CodecObject* self, PyObject* args, PyObject* kwds) {
  BEHOLDER_TRY { return codec_init_impl(self, args, kwds); }
  BEHOLDER_CATCH(-1)
}

int codec_init_impl(CodecObject* self, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"type_name", "fields", "dialect", nullptr};
  const char* tname;
  PyObject* fields;
  const char* dialect = "upb";
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "sO|s", const_cast<char**>(kwlist), &tname, &fields, &dialect))
    return -1;
  if (std::strcmp(dialect, "upb") == 0) {
    self->dialect = D_UPB;
  } else if (std::strcmp(dialect, "protobufjs") == 0) {
    self->dialect = D_PROTOBUFJS;
  } else {
    PyErr_Format(PyExc_ValueError, "unknown dialect %s (upb|protobufjs)", dialect);
    return -1;
  }
  PyObject* seq = PySequence_Fast(fields, "fields must be a sequence");
  if (!seq) return -1;
  Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  if (n < 1 || n > MAX_FIELDS) {
    Py_DECREF(seq);
    PyErr_Format(PyExc_ValueError, "MessageCodec supports 1..%d fields", MAX_FIELDS);
    return -1;
  }
  auto* specs = new std::vector<FieldSpec>();
  PyObject* names = PyTuple_New(n);
  PyObject* defaults = PyTuple_New(n);
  uint32_t max_no = 0;
  // PyStructSequence field names must outlive the type: they are copied into
  // heap memory that is intentionally never freed (codecs are created once per
  // message type per process).
  auto* members = static_cast<PyStructSequence_Field*>(PyMem_RawCalloc(size_t(n) + 1, sizeof(PyStructSequence_Field)));
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* item = PySequence_Fast_GET_ITEM(seq, i);
    unsigned long number;
    const char* fname;
    int kind;
    if (!PyArg_ParseTuple(item, "ksi", &number, &fname, &kind)) goto fail;
    if (number == 0 || number > MAX_FIELD_NUMBER) {
      PyErr_Format(PyExc_ValueError, "field number %lu out of range", number);
      goto fail;
    }
    if (kind < wire::K_STRING || kind > wire::K_SFIXED64) {
      PyErr_Format(PyExc_ValueError, "unknown field kind %d", kind);
      goto fail;
    }
    if (self->dialect == D_PROTOBUFJS && (kind == wire::K_INT64 || kind == wire::K_UINT64 || kind == wire::K_SINT64 ||
                                          kind == wire::K_FIXED64 || kind == wire::K_SFIXED64)) {
      // protobufjs returns Long objects for these; nothing in the telemetry schema uses them
      PyErr_Format(PyExc_ValueError, "protobufjs dialect does not model 64-bit integer field %s", fname);
      goto fail;
    }
    for (auto& s : *specs) {
      if (s.number == number) {
        PyErr_Format(PyExc_ValueError, "duplicate field number %lu", number);
        goto fail;
      }
    }
    specs->push_back(FieldSpec{uint32_t(number), kind});
    if (number > max_no) max_no = uint32_t(number);
    size_t L = strlen(fname);
    char* copy = static_cast<char*>(PyMem_RawMalloc(L + 1));
    memcpy(copy, fname, L + 1);
    members[i].name = copy;
    members[i].doc = nullptr;
    PyTuple_SET_ITEM(names, i, PyUnicode_FromString(fname));
    PyTuple_SET_ITEM(defaults, i, default_for(kind));
  }
  {
    size_t tl = strlen(tname);
    char* tcopy = static_cast<char*>(PyMem_RawMalloc(tl + 1));
    memcpy(tcopy, tname, tl + 1);
    auto* desc = static_cast<PyStructSequence_Desc*>(PyMem_RawCalloc(1, sizeof(PyStructSequence_Desc)));
    desc->name = tcopy;
    desc->doc = "decoded protobuf message (native codec)";
    desc->fields = members;
    desc->n_in_sequence = int(n);
    PyTypeObject* rt = PyStructSequence_NewType(desc);
    if (!rt) goto fail;
    self->result_type = rt;
    self->fast_new = type_size_attr(rt, "n_fields") == n && type_size_attr(rt, "n_sequence_fields") == n &&
                     type_size_attr(rt, "n_unnamed_fields") == 0 && rt->tp_itemsize == sizeof(PyObject*);
    if (self->fast_new) rt->tp_dealloc = result_dealloc;
    PyErr_Clear();
  }
  self->by_number = new std::vector<int16_t>(size_t(max_no) + 1, int16_t(-1));
  for (size_t i = 0; i < specs->size(); ++i) (*self->by_number)[(*specs)[i].number] = int16_t(i);
  self->fields = specs;
  self->names = names;
  self->defaults = defaults;
  self->type_name = PyUnicode_FromString(tname);
  Py_DECREF(seq);
  return 0;
fail:
  delete specs;
  Py_DECREF(names);
  Py_DECREF(defaults);
  Py_DECREF(seq);
  return -1;
}

inline PyObject* raise_decode(const char* why, PyObject* tname) {
  PyErr_Format(g_state.decode_error ? g_state.decode_error : PyExc_ValueError,
               "invalid wire format for %U: %s", tname, why);
  return nullptr;
}

// Core decode: fills `vals`/`seen`. Returns nullptr on success, else error text.
const char* decode_into(CodecObject* self, const uint8_t* data, size_t len, SlotVal* vals, bool* seen) {
  wire::Reader r(data, len);
  const auto& bynum = *self->by_number;
  const auto& specs = *self->fields;
  while (!r.eof()) {
    uint64_t tag;
    if (!r.tag(&tag)) return r.err;
    uint32_t field = uint32_t(tag >> 3);
    uint32_t wt = uint32_t(tag & 7);
    if (field == 0) return "invalid field number 0";
    int slot = field < bynum.size() ? bynum[field] : -1;
    if (slot < 0 || wire::expected_wire_type(specs[slot].kind) != wt) {
      if (!r.skip(wt, field)) return r.err;
      continue;
    }
    SlotVal& v = vals[slot];
    switch (wt) {
      case wire::WT_VARINT:
        if (!r.varint(&v.u)) return r.err;
        break;
      case wire::WT_LEN:
        if (!r.bytes(&v.s.p, &v.s.n)) return r.err;
        break;
      case wire::WT_I32: {
        uint32_t x;
        if (!r.fixed32(&x)) return r.err;
        v.u = x;
        break;
      }
      case wire::WT_I64:
        if (!r.fixed64(&v.u)) return r.err;
        break;
    }
    seen[slot] = true;
  }
  return nullptr;
}

// protobufjs dialect (pbjs.hpp): the generated decoder's loop. Values are final (already
// narrowed as protobufjs narrows them); strings hold their clamped byte range.
bool decode_pbjs_into(CodecObject* self, pbjs::Reader& r, SlotVal* vals, bool* seen) {
  const auto& bynum = *self->by_number;
  const auto& specs = *self->fields;
  while (r.pos < r.len) {
    uint32_t t;
    if (!r.uint32(&t)) return false;
    uint32_t field = t >> 3;
    int slot = field < bynum.size() ? bynum[field] : -1;
    if (slot < 0) {
      if (!r.skip_type(t & 7)) return false;
      continue;
    }
    SlotVal& v = vals[slot];
    switch (specs[slot].kind) {
      case wire::K_STRING:
        if (!r.string(&v.s.p, &v.s.n)) return false;
        break;
      case wire::K_BYTES:
        if (!r.bytes(&v.s.p, &v.s.n)) return false;
        break;
      case wire::K_FLOAT:
      case wire::K_FIXED32:
      case wire::K_SFIXED32: {
        uint32_t x;
        if (!r.fixed32(&x)) return false;
        v.u = x;
        break;
      }
      case wire::K_DOUBLE:
        if (!r.fixed64(&v.u)) return false;
        break;
      default: {  // int32 / enum / uint32 / sint32 / bool: Reader.uint32() and its narrowing
        uint32_t x;
        if (!r.uint32(&x)) return false;
        v.u = x;
        break;
      }
    }
    seen[slot] = true;
  }
  return true;
}

PyObject* value_for(int kind, const SlotVal& v) {
  switch (kind) {
    case wire::K_STRING:
      return PyUnicode_DecodeUTF8(reinterpret_cast<const char*>(v.s.p), Py_ssize_t(v.s.n), "strict");
    case wire::K_BYTES:
      return PyBytes_FromStringAndSize(reinterpret_cast<const char*>(v.s.p), Py_ssize_t(v.s.n));
    case wire::K_INT32:
    case wire::K_ENUM:
      return PyLong_FromLong(long(int32_t(uint32_t(v.u))));
    case wire::K_INT64:
      return PyLong_FromLongLong(int64_t(v.u));
    case wire::K_UINT32:
      return PyLong_FromUnsignedLong(uint32_t(v.u));
    case wire::K_UINT64:
      return PyLong_FromUnsignedLongLong(v.u);
    case wire::K_SINT32:
      return PyLong_FromLong(wire::unzigzag32(uint32_t(v.u)));
    case wire::K_SINT64:
      return PyLong_FromLongLong(wire::unzigzag64(v.u));
    case wire::K_BOOL:
      return PyBool_FromLong(v.u != 0);
    case wire::K_FLOAT: {
      uint32_t b = uint32_t(v.u);
      float f;
      memcpy(&f, &b, 4);
      return PyFloat_FromDouble(double(f));
    }
    case wire::K_DOUBLE: {
      double d;
      memcpy(&d, &v.u, 8);
      return PyFloat_FromDouble(d);
    }
    case wire::K_FIXED32:
      return PyLong_FromUnsignedLong(uint32_t(v.u));
    case wire::K_FIXED64:
      return PyLong_FromUnsignedLongLong(v.u);
    case wire::K_SFIXED32:
      return PyLong_FromLong(int32_t(uint32_t(v.u)));
    case wire::K_SFIXED64:
      return PyLong_FromLongLong(int64_t(v.u));
  }
  Py_RETURN_NONE;
}

}  // namespace

// Decodes `data` with codec `self_obj`; used by MessageCodec.decode.
PyObject* codec_decode_raw(PyObject* self_obj, const uint8_t* data, size_t len) {
  CodecObject* self = reinterpret_cast<CodecObject*>(self_obj);
  const size_t n = self->fields->size();
  SlotVal vals[MAX_FIELDS];
  bool seen[MAX_FIELDS] = {false};
  const bool pbjs_dialect = self->dialect == D_PROTOBUFJS;
  if (pbjs_dialect) {
    pbjs::Reader r(data, len);
    if (!decode_pbjs_into(self, r, vals, seen)) {
      // protobufjs's own message: it is what `err.message` logs (index.js:150)
      PyErr_SetString(g_state.decode_error ? g_state.decode_error : PyExc_ValueError, r.err);
      return nullptr;
    }
  } else {
    const char* err = decode_into(self, data, len, vals, seen);
    if (err) return raise_decode(err, self->type_name);
  }
  PyObject* out = new_result(self, Py_ssize_t(n));
  if (!out) return nullptr;
  for (size_t i = 0; i < n; ++i) {
    PyObject* v;
    if (seen[i]) {
      const int kind = (*self->fields)[i].kind;
      v = pbjs_dialect && (kind == wire::K_STRING) ? PyUnicode_DecodeUTF8(reinterpret_cast<const char*>(vals[i].s.p),
                                                                          Py_ssize_t(vals[i].s.n), "replace")
                                                   : value_for(kind, vals[i]);
      if (!v) {
        Py_DECREF(out);
        if (PyErr_ExceptionMatches(PyExc_UnicodeDecodeError)) {
          PyErr_Clear();
          return raise_decode("string field contains invalid UTF-8", self->type_name);
        }
        return nullptr;
      }
    } else {
      v = PyTuple_GET_ITEM(self->defaults, Py_ssize_t(i));
      Py_INCREF(v);
    }
    PyStructSequence_SET_ITEM(out, Py_ssize_t(i), v);
  }
  return out;
}

namespace {

PyObject* codec_decode(CodecObject* self, PyObject* arg) {
  if (PyBytes_CheckExact(arg)) {
    return codec_decode_raw(reinterpret_cast<PyObject*>(self),
                            reinterpret_cast<const uint8_t*>(PyBytes_AS_STRING(arg)),
                            size_t(PyBytes_GET_SIZE(arg)));
  }
  Py_buffer view;
  if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) < 0) {
    PyErr_Clear();
    PyErr_Format(g_state.decode_error ? g_state.decode_error : PyExc_ValueError,
                 "illegal buffer: expected bytes-like, got %s", Py_TYPE(arg)->tp_name);
    return nullptr;
  }
  PyObject* out = codec_decode_raw(reinterpret_cast<PyObject*>(self),
                                   static_cast<const uint8_t*>(view.buf), size_t(view.len));
  PyBuffer_Release(&view);
  return out;
}

// Encode a value for `kind`; appends to `buf`. Returns false with Python error set.
bool encode_field(std::string& buf, uint32_t number, int kind, PyObject* v) {
  using namespace wire;
  uint8_t tmp[16];
  auto put_tag = [&](uint32_t wt) {
    uint8_t* e = put_varint(tmp, (uint64_t(number) << 3) | wt);
    buf.append(reinterpret_cast<char*>(tmp), size_t(e - tmp));
  };
  auto put_v = [&](uint64_t x) {
    uint8_t* e = put_varint(tmp, x);
    buf.append(reinterpret_cast<char*>(tmp), size_t(e - tmp));
  };
  switch (kind) {
    case K_STRING: {
      Py_ssize_t L;
      const char* s = PyUnicode_AsUTF8AndSize(v, &L);
      if (!s) return false;
      if (L == 0) return true;
      put_tag(WT_LEN);
      put_v(uint64_t(L));
      buf.append(s, size_t(L));
      return true;
    }
    case K_BYTES: {
      char* s;
      Py_ssize_t L;
      if (PyBytes_AsStringAndSize(v, &s, &L) < 0) return false;
      if (L == 0) return true;
      put_tag(WT_LEN);
      put_v(uint64_t(L));
      buf.append(s, size_t(L));
      return true;
    }
    case K_FLOAT:
    case K_DOUBLE: {
      double d = PyFloat_AsDouble(v);
      if (d == -1.0 && PyErr_Occurred()) return false;
      if (d == 0.0 && !std::signbit(d)) return true;
      if (kind == K_FLOAT) {
        float f = float(d);
        put_tag(WT_I32);
        buf.append(reinterpret_cast<char*>(&f), 4);
      } else {
        put_tag(WT_I64);
        buf.append(reinterpret_cast<char*>(&d), 8);
      }
      return true;
    }
    case K_BOOL: {
      int t = PyObject_IsTrue(v);
      if (t < 0) return false;
      if (!t) return true;
      put_tag(WT_VARINT);
      put_v(1);
      return true;
    }
    default:
      break;
  }
  // integer kinds
  int overflow = 0;
  long long sv = PyLong_AsLongLongAndOverflow(v, &overflow);
  uint64_t uv;
  if (sv == -1 && PyErr_Occurred()) return false;
  if (overflow > 0) {
    uv = PyLong_AsUnsignedLongLong(v);
    if (PyErr_Occurred()) return false;
    sv = int64_t(uv);
  } else if (overflow < 0) {
    PyErr_SetString(PyExc_OverflowError, "integer out of range");
    return false;
  } else {
    uv = uint64_t(sv);
  }
  if (uv == 0) return true;
  switch (kind) {
    case K_INT32:
    case K_ENUM:
      put_tag(WT_VARINT);
      put_v(uint64_t(int64_t(int32_t(sv))));  // negative int32 -> 10-byte varint
      return true;
    case K_UINT32:
      put_tag(WT_VARINT);
      put_v(uint32_t(uv));
      return true;
    case K_INT64:
    case K_UINT64:
      put_tag(WT_VARINT);
      put_v(uv);
      return true;
    case K_SINT32:
      put_tag(WT_VARINT);
      put_v(zigzag32(int32_t(sv)));
      return true;
    case K_SINT64:
      put_tag(WT_VARINT);
      put_v(zigzag64(sv));
      return true;
    case K_FIXED32:
    case K_SFIXED32: {
      uint32_t x = uint32_t(uv);
      put_tag(WT_I32);
      buf.append(reinterpret_cast<char*>(&x), 4);
      return true;
    }
    case K_FIXED64:
    case K_SFIXED64:
      put_tag(WT_I64);
      buf.append(reinterpret_cast<char*>(&uv), 8);
      return true;
  }
  PyErr_SetString(PyExc_ValueError, "bad kind");
  return false;
}

// encode(obj) where obj is a sequence in slot order or a mapping by field name.
PyObject* codec_encode_impl(CodecObject* self, PyObject* obj);
PyObject* codec_encode(CodecObject* self, PyObject* obj) {
  BEHOLDER_TRY { return codec_encode_impl(self, obj); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* codec_encode_impl(CodecObject* self, PyObject* obj) {
  const size_t n = self->fields->size();
  std::string buf;
  buf.reserve(64);
  bool is_map = PyDict_Check(obj);
  PyObject* seq = nullptr;
  if (!is_map) {
    seq = PySequence_Fast(obj, "encode() takes a mapping or a sequence in field order");
    if (!seq) return nullptr;
    if (size_t(PySequence_Fast_GET_SIZE(seq)) != n) {
      Py_DECREF(seq);
      PyErr_Format(PyExc_ValueError, "expected %zu values", n);
      return nullptr;
    }
  }
  for (size_t i = 0; i < n; ++i) {
    PyObject* v;
    if (is_map) {
      v = PyDict_GetItemWithError(obj, PyTuple_GET_ITEM(self->names, Py_ssize_t(i)));
      if (!v) {
        if (PyErr_Occurred()) return nullptr;
        continue;
      }
    } else {
      v = PySequence_Fast_GET_ITEM(seq, Py_ssize_t(i));
    }
    if (v == Py_None) continue;
    const FieldSpec& f = (*self->fields)[i];
    if (!encode_field(buf, f.number, f.kind, v)) {
      Py_XDECREF(seq);
      return nullptr;
    }
  }
  Py_XDECREF(seq);
  return PyBytes_FromStringAndSize(buf.data(), Py_ssize_t(buf.size()));
}

PyObject* codec_get_result_type(CodecObject* self, void*) {
  Py_INCREF(self->result_type);
  return reinterpret_cast<PyObject*>(self->result_type);
}
PyObject* codec_get_names(CodecObject* self, void*) {
  Py_INCREF(self->names);
  return self->names;
}
PyObject* codec_get_type_name(CodecObject* self, void*) {
  Py_INCREF(self->type_name);
  return self->type_name;
}
PyObject* codec_get_dialect(CodecObject* self, void*) {
  return PyUnicode_FromString(self->dialect == D_PROTOBUFJS ? "protobufjs" : "upb");
}

PyMethodDef codec_methods[] = {
    {"decode", reinterpret_cast<PyCFunction>(codec_decode), METH_O,
     "decode(data) -> message; raises DecodeError on malformed input"},
    {"encode", reinterpret_cast<PyCFunction>(codec_encode), METH_O,
     "encode(mapping_or_sequence) -> bytes (proto3: default values omitted)"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef codec_getset[] = {
    {"result_type", reinterpret_cast<getter>(codec_get_result_type), nullptr, "decoded message type", nullptr},
    {"field_names", reinterpret_cast<getter>(codec_get_names), nullptr, "field names in slot order", nullptr},
    {"type_name", reinterpret_cast<getter>(codec_get_type_name), nullptr, "message type name", nullptr},
    {"dialect", reinterpret_cast<getter>(codec_get_dialect), nullptr, "decode dialect: upb | protobufjs", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

// materialise_table(buf, table) -> [(mediaId, status, progress, host), ...]
// Host half of the GPU-offload probe (ops/gpu_decode.py): turns the kernel's (n, 8) int32 field
// table back into the Python values the handlers use. Rows with ok == 0 give None. Offsets are
// re-checked against len(buf): the table comes from a device and is not trusted.
PyObject* mod_materialise_table(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 2) {
    PyErr_SetString(PyExc_TypeError, "materialise_table(buf, table)");
    return nullptr;
  }
  Py_buffer b, t;
  if (PyObject_GetBuffer(a[0], &b, PyBUF_SIMPLE) < 0) return nullptr;
  if (PyObject_GetBuffer(a[1], &t, PyBUF_FORMAT | PyBUF_C_CONTIGUOUS) < 0) {
    PyBuffer_Release(&b);
    return nullptr;
  }
  PyObject* out = nullptr;
  if (t.itemsize != 4 || t.len % 32 != 0) {
    PyErr_SetString(PyExc_TypeError, "table must be a contiguous (n, 8) int32 buffer");
  } else {
    const Py_ssize_t rows = t.len / 32;
    const int32_t* tab = static_cast<const int32_t*>(t.buf);
    const char* base = static_cast<const char*>(b.buf);
    out = PyList_New(rows);
    for (Py_ssize_t k = 0; out && k < rows; ++k) {
      const int32_t* r = tab + 8 * k;
      PyObject* item;
      if (!r[6]) {
        item = Py_NewRef(Py_None);
      } else if (r[0] < 0 || r[1] < 0 || r[4] < 0 || r[5] < 0 || r[0] + int64_t(r[1]) > b.len ||
                 r[4] + int64_t(r[5]) > b.len) {
        PyErr_Format(PyExc_ValueError, "row %zd points outside the batch", k);
        item = nullptr;
      } else {
        PyObject* id = PyUnicode_DecodeUTF8(base + r[0], r[1], "replace");
        PyObject* host = PyUnicode_DecodeUTF8(base + r[4], r[5], "replace");
        PyObject* st = PyLong_FromLong(r[2]);
        PyObject* pr = PyLong_FromLong(r[3]);
        item = (id && host && st && pr) ? PyTuple_Pack(4, id, st, pr, host) : nullptr;
        Py_XDECREF(id);
        Py_XDECREF(host);
        Py_XDECREF(st);
        Py_XDECREF(pr);
      }
      if (!item) {
        Py_CLEAR(out);
        break;
      }
      PyList_SET_ITEM(out, k, item);
    }
  }
  PyBuffer_Release(&t);
  PyBuffer_Release(&b);
  return out;
}

PyMethodDef codec_functions[] = {
    {"materialise_table", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(mod_materialise_table)),
     METH_FASTCALL, "materialise_table(buf, table) -> list of (mediaId, status, progress, host) or None"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

PyTypeObject CodecType = {PyVarObject_HEAD_INIT(nullptr, 0)};

int init_codec_types(PyObject* m) {
  CodecType.tp_name = "beholder_amd.ops._native.MessageCodec";
  CodecType.tp_basicsize = sizeof(CodecObject);
  CodecType.tp_flags = Py_TPFLAGS_DEFAULT;
  CodecType.tp_doc = "MessageCodec(type_name, fields): native protobuf codec for flat messages";
  CodecType.tp_new = codec_new;
  CodecType.tp_init = reinterpret_cast<initproc>(codec_init);
  CodecType.tp_dealloc = reinterpret_cast<destructor>(codec_dealloc);
  CodecType.tp_methods = codec_methods;
  CodecType.tp_getset = codec_getset;
  if (PyType_Ready(&CodecType) < 0) return -1;
  Py_INCREF(&CodecType);
  if (PyModule_AddObject(m, "MessageCodec", reinterpret_cast<PyObject*>(&CodecType)) < 0) return -1;
  return PyModule_AddFunctions(m, codec_functions);
}

}  // namespace beholder
