// Read-only safetensors checkpoint (single file or a sharded *.index.json), memory-mapped.
// The stage loader (bs_init_stage_file, stage.hip) takes each tensor of its layer range straight from
// the mapping: only the pages of the stage's own tensors are ever read, and no fp32 copy of the
// model is built on the host (BS_WEIGHTS_HOST needs one: ~28 GB for bloom-7b1).
#pragma once
#include <cstddef>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace st {

enum Dtype { F32 = 0, F16 = 1, BF16 = 2, OTHER = 3 };

struct Tensor {
  Dtype dtype = OTHER;
  std::string dtype_name;
  std::vector<int64_t> shape;
  const uint8_t* data = nullptr;  // inside the file mapping
  uint64_t bytes = 0;
  uint64_t numel() const {
    uint64_t n = 1;
    for (int64_t d : shape) n *= (uint64_t)d;
    return n;
  }
};

class Checkpoint {
 public:
  ~Checkpoint();
  // path: a .safetensors file or a sharded checkpoint's index JSON ({"weight_map": {name: file}}).
  // Returns false with *err set on a malformed or truncated file.
  bool open(const std::string& path, std::string* err);
  // Tensor by HF name; also tries the "transformer." prefix of BloomForCausalLM checkpoints.
  const Tensor* find(const std::string& name) const;
  const std::map<std::string, Tensor>& tensors() const { return tensors_; }

 private:
  bool map_file(const std::string& path, std::string* err);
  struct Mapping { void* base; size_t len; };
  std::vector<Mapping> maps_;
  std::map<std::string, Tensor> tensors_;
};

}  // namespace st
