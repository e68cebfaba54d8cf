"""``Net(upscale_factor)`` -- the super-resolution CNN of Fairscale-DDP.py:74 (module ``models.sr_4k_2x``,
absent from the reference, SURVEY.md F1: contract [B,3,H,W] -> [B,3,rH,rW]).  Re-created as an
ESPCN-style sub-pixel network (conv 5x5 64 -> conv 3x3 64 -> conv 3x3 32 -> conv 3x3 3r^2 -> PixelShuffle);
the exact upstream layer sizes are unknown ("parity unpinned"), the I/O contract is the reference's."""
import torch.nn as nn


class Net(nn.Module):
    def __init__(self, upscale_factor: int = 2, in_chans: int = 3, width: int = 64):
        super().__init__()
        r = upscale_factor
        self.body = nn.Sequential(
            nn.Conv2d(in_chans, width, 5, padding=2), nn.Tanh(),
            nn.Conv2d(width, width, 3, padding=1), nn.Tanh(),
            nn.Conv2d(width, width // 2, 3, padding=1), nn.Tanh(),
            nn.Conv2d(width // 2, in_chans * r * r, 3, padding=1),
        )
        self.shuffle = nn.PixelShuffle(r)
        self.up = nn.Upsample(scale_factor=r, mode="bilinear", align_corners=False)

    def forward(self, x):
        # global residual on a bilinear upsample keeps early training stable
        return self.up(x) + self.shuffle(self.body(x))
