"""mipipe: MI355X-native pipeline-parallel LLM inference engine (package `distributed-llm-pipeline_amd`).

Layout:
  models/    model configs, synthetic GGUF generator, pure-torch reference model (oracle)
  ops/       torch wrappers of the hand-written gfx950 HIP kernels (tests / tools)
  parallel/  engine + pipeline front-end (stage partitioner, torch.distributed rendezvous)
  utils/     GGUF v3 writer/reader, ggml quant reference implementations
Native code lives in `csrc/` (HIP kernels + C++ runtime) and is built into `lib/libmipipe.so`.
"""
__version__ = "0.1.0"
