"""CPU oracle — TEST INFRASTRUCTURE ONLY.

A plain restatement of the reference's algorithms for the hot path
(qazi0/real-time-disaster-management, paths under /root/reference/code):
  classifier.py  ACFF models (disaster_detection/model/*.py) in torch-CPU fp32
  darknet.py     cfg-driven Darknet forward + YOLOLayer decode (yolov3/models.py)
  nms.py         non_max_suppression (yolov3/utils/utils.py:488-557) + the
                 torchvision.ops.boxes.nms CPU kernel it calls (numpy)
  preprocess.py  the classifier CLI transform (dataloaders/aider.py:412-426):
                 Pillow 8-bit antialiased bilinear resize restated in numpy
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / CPU baseline — never as the product path.

Pinning (see DESIGN.md "Oracle"): classifier, darknet and the non-NMS parts of
non_max_suppression are pinned against golden vectors produced by the
reference code itself (tests/golden/make_golden.py); the preprocess restatement
is pinned against Pillow; the torchvision NMS kernel (third-party, absent) is a
restatement of torchvision 0.8.2's CPU nms_kernel — parity unpinned at that
boundary.
"""
