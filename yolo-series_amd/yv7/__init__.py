"""yv7 — the MI355X-native runtime behind the reference's models.yolo / utils.general API.

  yv7.arch       yolov7 / yolov7-tiny / yolov7-w6 graph definitions (reference cfg schema)
  yv7.graph      Model -> flat plan (NHWC tensors, ops, packed weights)
  yv7.runtime    Plan: the compiled network on one GPU, driven through libyv7.so (C ABI, include/yv7.h)
  yv7.synthetic  seeded synthetic weights / frames (no checkpoints offline)
  yv7.dist       batch sharding over the GPUs of a node (RCCL broadcast of weights, all-gather of detections)
"""
