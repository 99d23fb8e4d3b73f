// Minimal protobuf wire-format codec for the TensorFlow GraphDef subset used by
// TensorFrames: GraphDef / NodeDef / AttrValue / TensorProto / TensorShapeProto.
//
// There is no protoc/libprotobuf in this environment, so the messages are
// decoded directly from the wire format. Field numbers follow
// reference: src/main/protobuf/tensorflow/core/framework/graph.proto:14-112,
// attr_value.proto:16-60, tensor.proto:13-60, tensor_shape.proto:12-45.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../common.h"

namespace tfa {

// Host-side decoded tensor (TensorProto). Numeric payload is stored densely in
// little-endian `bytes`; string tensors use `strings`.
struct HostTensor {
  DType dtype = DType::INVALID;
  Shape shape;
  std::vector<uint8_t> bytes;
  std::vector<std::string> strings;

  int64_t num_elements() const { return shape.num_elements(); }
  template <typename T>
  const T* as() const { return reinterpret_cast<const T*>(bytes.data()); }
  template <typename T>
  T* as_mut() { return reinterpret_cast<T*>(bytes.data()); }
  // Reads element i as a double / int64 regardless of dtype (for attrs & folding).
  double get_f(int64_t i) const;
  int64_t get_i(int64_t i) const;
};

struct AttrValue;

struct AttrList {
  std::vector<std::string> s;
  std::vector<int64_t> i;
  std::vector<float> f;
  std::vector<bool> b;
  std::vector<DType> type;
  std::vector<Shape> shape;
  std::vector<HostTensor> tensor;
};

struct AttrValue {
  enum Kind { NONE, LIST, S, I, F, B, TYPE, SHAPE, TENSOR, PLACEHOLDER, FUNC } kind = NONE;
  std::string s;  // also placeholder / func name
  int64_t i = 0;
  float f = 0.f;
  bool b = false;
  DType type = DType::INVALID;
  Shape shape;
  std::shared_ptr<HostTensor> tensor;
  std::shared_ptr<AttrList> list;
};

struct NodeDef {
  std::string name;
  std::string op;
  std::vector<std::string> inputs;
  std::string device;
  std::map<std::string, AttrValue> attr;

  const AttrValue* find_attr(const std::string& k) const {
    auto it = attr.find(k);
    return it == attr.end() ? nullptr : &it->second;
  }
};

struct GraphDef {
  std::vector<NodeDef> nodes;
  int producer = 0;
};

// upper bound on one decoded constant's bytes (env TFA_MAX_CONST_BYTES, default 64 GiB)
int64_t max_constant_bytes();
GraphDef parse_graphdef(const std::string& bytes);
HostTensor parse_tensor_proto(const std::string& bytes);
Shape parse_shape_proto(const std::string& bytes);

std::string serialize_graphdef(const GraphDef& g);
std::string serialize_tensor_proto(const HostTensor& t);

}  // namespace tfa
