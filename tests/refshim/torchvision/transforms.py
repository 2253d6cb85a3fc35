"""torchvision.transforms subset with torchvision's tensor semantics (see __init__)."""
import torch


class Compose:
    def __init__(self, ts):
        self.ts = ts

    def __call__(self, x):
        for t in self.ts:
            x = t(x)
        return x


class ToTensor:
    """uint8 HxW image -> float32 [1,H,W] in [0,1] (torchvision: .float().div(255))."""

    def __call__(self, img):
        return img.unsqueeze(0).contiguous().to(dtype=torch.get_default_dtype()).div(255)


class Normalize:
    """(x - mean) / std per channel (torchvision: sub_(mean[:,None,None]).div_(std[:,None,None]))."""

    def __init__(self, mean, std):
        self.mean, self.std = mean, std

    def __call__(self, t):
        mean = torch.as_tensor(self.mean, dtype=t.dtype)
        std = torch.as_tensor(self.std, dtype=t.dtype)
        return t.clone().sub_(mean[:, None, None]).div_(std[:, None, None])
