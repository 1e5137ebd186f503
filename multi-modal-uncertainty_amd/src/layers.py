"""Conv blocks of the FashionMNIST MIMO ResNet (BASELINE config 1: CPU plumbing).

Drop-in for the working part of the reference src/layers.py: ``BasicBlock``
(src/layers.py:7-39).  The reference file's ``OutputLayer`` redefinitions refer to
undefined names (src/layers.py:109-149) and are not reproduced.  The
modality-token concat / gather the north star places "in src/layers.py" lives in
src/mmbt.py in the reference and in the HIP embedding kernel here (csrc/embed.hip).
"""
import torch.nn as nn


def conv3x3(in_planes, out_planes, stride=1):
    """3x3 conv, padding 1, no bias (torchvision.models.resnet.conv3x3, src/layers.py:4)."""
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=False)


class BasicBlock(nn.Module):
    """src/layers.py:7-39: conv-bn-relu-conv-bn (+ downsample skip), relu.  Child names and
    registration order (relu, bn1, conv1, bn2, conv2, downsample) follow the reference so the
    state_dict keys match."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.relu = nn.ReLU(inplace=True)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv2 = conv3x3(planes, planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        skip = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return self.relu(y + skip)
