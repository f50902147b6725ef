"""Write the bench's base texture (synthetic.make_texture, 1080 x 1920 uint16, seed 0)
as a raw file for tools/warp_lab:  python tools/write_texture.py out.u16"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kcmc_amd import synthetic  # noqa: E402

synthetic.make_texture((1080, 1920), seed=0).astype("<u2").tofile(sys.argv[1])
