"""Reset-side inputs: the BinaryNet pre-model and the PNG
target loader that feed env.reset (env.py:96-120, DBS_1024_24.py:48-201).

``BinaryNet`` is the reference's U-Net-shaped pre-model rebuilt on torch.nn
(PyTorch-ROCm runs the convolutions on MIOpen): the same constructor switches
and the same sub-module names, so a reference checkpoint's state_dict loads
unchanged (``load_premodel`` uses ``torch.load(weights_only=True)``).  Every
"CRB" block is conv3x3 (+ Tanh) (+ BatchNorm), every "TRB" block a 2x2
stride-2 transposed conv (+ BatchNorm) (+ ReLU); the encoder halves the
resolution four times with stride-2 CRB blocks, the decoder concatenates the
skip connections; the classifier is a bare conv3x3 followed by a sigmoid.

``TargetFolder`` replaces the reference's ``Dataset512`` (torchvision is not
in this image): sorted ``*.png`` of a directory, read with PIL, resized so the
shorter side is at least IPS, then a random (training) or centre crop of
IPS x IPS plus optional zero padding; items are (target [1, C, IPS, IPS], path)
like the reference's loader (DBS_1024_24.py:175-201).
"""
from __future__ import annotations

import glob
import os
from typing import Callable, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

DEFAULT_CHANNELS = (32, 64, 128, 256, 512, 1024, 2048, 4096)   # DBS_1024_24.py:50


def _crb(cin: int, cout: int, stride: int = 1, act: bool = True, bn: bool = True) -> nn.Sequential:
    mods = [nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=True)]
    if act:
        mods.append(nn.Tanh())
    if bn:
        mods.append(nn.BatchNorm2d(cout))
    return nn.Sequential(*mods)


def _trb(cin: int, cout: int, act: bool = True, bn: bool = True) -> nn.Sequential:
    mods = [nn.ConvTranspose2d(cin, cout, kernel_size=2, stride=2, padding=0, bias=True)]
    if bn:
        mods.append(nn.BatchNorm2d(cout))
    if act:
        mods.append(nn.ReLU())
    return nn.Sequential(*mods)


class BinaryNet(nn.Module):
    """Pre-model: target [B, in_planes, H, W] -> per-plane probabilities
    [B, num_hologram, H, W] (H, W divisible by 16).  Module names follow
    DBS_1024_24.py:48-164 / env.py's model so checkpoints are interchangeable."""

    def __init__(self, num_hologram: int, final: str = "Sigmoid", in_planes: int = 3,
                 channels: Sequence[int] = DEFAULT_CHANNELS, convReLU: bool = True, convBN: bool = True,
                 poolReLU: bool = True, poolBN: bool = True, deconvReLU: bool = True, deconvBN: bool = True):
        super().__init__()
        c = list(channels)
        cv = dict(act=convReLU, bn=convBN)
        pl = dict(act=poolReLU, bn=poolBN)
        dc = dict(act=deconvReLU, bn=deconvBN)
        prev = in_planes
        for lvl in range(1, 5):                      # encoder levels 1..4 with a stride-2 "pool"
            w = c[lvl - 1]
            setattr(self, f"enc{lvl}_1", _crb(prev, w, **cv))
            setattr(self, f"enc{lvl}_2", _crb(w, w, **cv))
            setattr(self, f"pool{lvl}", _crb(w, w, stride=2, **pl))
            prev = w
        self.enc5_1 = _crb(c[3], c[4], **cv)
        self.enc5_2 = _crb(c[4], c[4], **cv)
        for lvl in range(4, 0, -1):                  # decoder: upsample, concat skip, two convs
            w_in, w = c[lvl], c[lvl - 1]
            setattr(self, f"deconv{lvl}", _trb(w_in, w, **dc))
            setattr(self, f"dec{lvl}_1", _crb(w_in, w, **cv))
            setattr(self, f"dec{lvl}_2", _crb(w, w, **cv))
        self.classifier = _crb(c[0], num_hologram, act=False, bn=False)
        self.final = final

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        skips = []
        h = x
        for lvl in range(1, 5):
            h = getattr(self, f"enc{lvl}_2")(getattr(self, f"enc{lvl}_1")(h))
            skips.append(h)
            h = getattr(self, f"pool{lvl}")(h)
        h = self.enc5_2(self.enc5_1(h))
        for lvl in range(4, 0, -1):
            h = torch.cat((getattr(self, f"deconv{lvl}")(h), skips[lvl - 1]), dim=1)
            h = getattr(self, f"dec{lvl}_2")(getattr(self, f"dec{lvl}_1")(h))
        return torch.sigmoid(self.classifier(h))


def reference_premodel(num_hologram: int = 24, in_planes: int = 3) -> BinaryNet:
    """The instantiation the reference scripts use: plain convolutions, no
    activations or batch norm (DBS_1024_24.py:167-169, env.py's model)."""
    return BinaryNet(num_hologram=num_hologram, in_planes=in_planes, convReLU=False, convBN=False,
                     poolReLU=False, poolBN=False, deconvReLU=False, deconvBN=False)


def load_premodel(path: str, num_hologram: int = 24, in_planes: int = 3,
                  device: Optional[torch.device] = None, **kw) -> BinaryNet:
    """BinaryNet with a reference checkpoint (state_dict, or a dict holding
    one under 'model' / 'state_dict'), loaded with weights_only=True."""
    m = BinaryNet(num_hologram=num_hologram, in_planes=in_planes, **kw) if kw else \
        reference_premodel(num_hologram, in_planes)
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict):
        for key in ("model", "state_dict", "model_state_dict"):
            if key in sd and isinstance(sd[key], dict):
                sd = sd[key]
                break
    sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
    m.load_state_dict(sd)
    m.eval()
    return m.to(device) if device is not None else m


def premodel_fn(model: nn.Module, dtype: torch.dtype = torch.float32) -> Callable:
    """pre_model_fn for HologramVecEnv: target [1, C, H, W] -> [1, CH, H, W]
    under torch.no_grad (env.py:109-111).  dtype=torch.bfloat16 runs the
    convolutions in bf16 (the binarisation threshold is 0.5, so only values
    within bf16 resolution of 0.5 can change the initial state)."""
    model.eval()

    def fn(target: torch.Tensor) -> torch.Tensor:
        with torch.no_grad():
            if dtype == torch.float32:
                return model(target.float())
            with torch.autocast(device_type=target.device.type, dtype=dtype):
                return model(target).float()
    return fn


def _imread(path: str, gray: bool = False) -> torch.Tensor:
    from PIL import Image
    img = Image.open(path).convert("L" if gray else "RGB")
    a = np.asarray(img, dtype=np.float32) / 255.0
    a = a[None] if gray else np.transpose(a, (2, 0, 1))
    return torch.from_numpy(np.ascontiguousarray(a))


class TargetFolder:
    """Sorted ``*.png`` targets of a directory.  ``ds[i]`` is (target [1, C, IPS, IPS], path);
    iterating yields what ``DataLoader(Dataset512(...), batch_size=1)`` yields, the batched
    target and the collated name LIST ``[path]`` (``a, imgname = next(iter(trainloader))``,
    DBS_1024_24.py:271; env.py:96-104 prints it), so it drops in for the reference's loader."""

    def __init__(self, target_dir: str, ips: int = 1024, train: bool = True, padding: int = 0,
                 gray: bool = False, seed: Optional[int] = None):
        self.target_list = sorted(glob.glob(os.path.join(target_dir, "*.png")))
        self.ips, self.train, self.padding, self.gray = int(ips), bool(train), int(padding), gray
        self.gen = torch.Generator().manual_seed(seed if seed is not None else 0)

    def __len__(self) -> int:
        return len(self.target_list)

    def _prepare(self, t: torch.Tensor) -> torch.Tensor:
        n = self.ips
        h, w = t.shape[-2:]
        if h < n or w < n:                            # smaller side -> IPS, aspect kept
            s = n / min(h, w)
            t = F.interpolate(t[None], size=(max(n, round(h * s)), max(n, round(w * s))),
                              mode="bilinear", align_corners=False, antialias=True)[0]
            h, w = t.shape[-2:]
        if self.train:
            y = int(torch.randint(0, h - n + 1, (1,), generator=self.gen))
            x = int(torch.randint(0, w - n + 1, (1,), generator=self.gen))
        else:                                          # torchvision CenterCrop rounding
            y, x = int(round((h - n) / 2.0)), int(round((w - n) / 2.0))
        t = t[:, y:y + n, x:x + n]
        if self.padding:
            p = self.padding
            t = F.pad(t, (p, p, p, p))
        return t

    def __getitem__(self, idx: int):
        path = self.target_list[idx]
        return self._prepare(_imread(path, self.gray))[None], path

    def __iter__(self):
        for i in range(len(self)):
            t, path = self[i]
            yield t, [path]
