"""ResNet-152 v1.5 image trunk (the torchvision module tree src/mmbt.py:19-21 slices).

Child order and parameter names follow torchvision's resnet152 so that
``ImageEncoder.model = Sequential(children[:-2])`` yields the reference keys
``enc.img_encoder.model.{0..7}.*``.  No pretrained weights exist offline: weights
use torchvision's default init (He-normal fan_out convs, BN gamma 1 / beta 0).
On MI355X the trunk runs through MIOpen in bf16, channels-last (ImageEncoder).
"""
import torch
import torch.nn as nn


class BatchNorm2d(nn.BatchNorm2d):
    """BatchNorm2d with two MI355X-specific forms (state_dict / semantics unchanged):
    * inference: a per-channel affine y = x * s + t (s = w / sqrt(var + eps),
      t = b - mean * s) in the activation dtype -- one elementwise pass;
    * training: MIOpen's batch-statistics kernels for real batches, PyTorch's native
      NHWC kernels below MIOPEN_MIN_BATCH images.
    On this ROCm 7.2 stack MIOpen's bf16 NHWC batch-norm crashes in host code for tiny
    batches (B=2 in training; inference), while the native kernels are ~2x slower at
    B=256 ("ResNet trunk")."""

    MIOPEN_MIN_BATCH = 8

    def forward(self, x):
        if self.training or not self.track_running_stats:
            with torch.backends.cudnn.flags(enabled=x.shape[0] >= self.MIOPEN_MIN_BATCH):
                return super().forward(x)
        s = self.weight * (self.running_var + self.eps).rsqrt()
        t = self.bias - self.running_mean * s
        return x * s.view(1, -1, 1, 1).to(x.dtype) + t.view(1, -1, 1, 1).to(x.dtype)


class Bottleneck(nn.Module):
    def __init__(self, cin, width, stride):
        super().__init__()
        cout = width * 4
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride, bias=False), BatchNorm2d(cout))

    def forward(self, x):
        skip = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        return self.relu(self.bn3(self.conv3(y)) + skip)


def resnet152_trunk(blocks=(3, 8, 36, 3)):
    """Sequential(conv1, bn1, relu, maxpool, layer1..layer4) -> [B,2048,H/32,W/32]."""
    mods = [nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False), BatchNorm2d(64), nn.ReLU(inplace=True),
            nn.MaxPool2d(3, 2, 1)]
    cin = 64
    for i, (width, n) in enumerate(zip((64, 128, 256, 512), blocks)):
        stage = []
        for b in range(n):
            stage.append(Bottleneck(cin, width, 2 if (b == 0 and i > 0) else 1))
            cin = width * 4
        mods.append(nn.Sequential(*stage))
    trunk = nn.Sequential(*mods)
    for m in trunk.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)
    return trunk
