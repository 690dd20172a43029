"""Write the package's data assets from the reference's own data files (run in the build
container only; /root/reference does not exist on the GPU box):

    python tools/make_assets.py

  siren_mri_amd/assets/irdata.npz   data/IRData.mat (the only MRI image data in the reference tree,
                                    read by MRIImageDomain, dataio.py:507-525): IRData [128, 128, 9]
                                    float32 magnitude slices (the singleton coil axis squeezed, as
                                    the reference's np.squeeze does) and TI [9] inversion times.
The cameraman (camera512_u8.npz) is written by tests/golden/make_golden.py.
Only data moves: no reference source is read or copied.
"""
import os

import numpy as np
import scipy.io as sio

REF = "/root/reference/data/IRData.mat"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "siren_mri_amd", "assets")


def main():
    m = sio.loadmat(REF)
    ir = np.ascontiguousarray(np.squeeze(m["IRData"]).astype(np.float32))
    ti = np.asarray(m["TI"], dtype=np.float64).reshape(-1)
    assert ir.shape == (128, 128, 9), ir.shape
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, "irdata.npz"), IRData=ir, TI=ti)
    print("wrote", os.path.join(OUT, "irdata.npz"), ir.shape, float(ir.min()), float(ir.max()))


if __name__ == "__main__":
    main()
