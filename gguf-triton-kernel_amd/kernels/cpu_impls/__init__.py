"""Drop-in for the reference's `kernels.cpu_impls` package: the CPU MMQ products with the
reference's exact arithmetic (fp16 running sum in block order), run by libgguf_quant.so
(csrc/quant/gguf_cpu_mmq.cpp, multithreaded C++).  Host tensors only; the GPU entry points
in `kernels.mmq_*` never call these."""
