"""Calibration of the synthetic image task on one MI355X: ResNet-18 validation accuracy over an
lr x epochs grid (the task must not saturate, and lr / epochs must move the accuracy)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from katib_amd.workloads import resnet_cifar  # noqa: E402

for lr in (0.01, 0.1, 0.4):
    a = resnet_cifar.main(["--epochs", "4", "--lr", str(lr), "--num-train", "20000", "--num-valid", "5000"])
    print("CALIB resnet lr", lr, "final", a, flush=True)
