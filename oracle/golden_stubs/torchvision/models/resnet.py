"""torchvision.models.resnet.conv3x3 stand-in (imported by the reference src/layers.py:4,
which src/model.py imports): the 3x3, padding-1, bias-free convolution."""
import torch.nn as nn


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation, groups=groups,
                     bias=False, dilation=dilation)
