"""Model families used by benchmarks, examples and tests (random init only).

* ``llama``  -- Llama-3 8B/70B geometry, FSDP2 builder (BASELINE configs 2, 3, 5)
* ``resnet`` -- ResNet-18 written by hand (torchvision is absent; BASELINE config 1)
* ``dlrm``   -- DLRM-style model with row-wise sharded embedding tables,
  optionally on managed (UVM) memory (BASELINE config 4)
* ``ddp_bench`` -- the reference's DDP benchmark model (N x 100 MB fp32 params)
"""
