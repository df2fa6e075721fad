"""Copies the reference's bundled AIDER / ODDER JPEGs (the inputs cv2.imread decodes in
victim_localization/yolov3/utils/datasets.py:97) into tests/golden/jpeg/ as decode
fixtures (data files, unique by content).  Run in the build container, where
/root/reference exists; the GPU box uses the committed copies.  The expected outputs are
Pillow's decode of each file (the same libjpeg-turbo defaults cv2 uses), computed by the
tests themselves."""
import glob
import hashlib
import os
import shutil

REF = "/root/reference/code/victim_localization"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "jpeg")

if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    seen = set()
    for f in sorted(glob.glob(f"{REF}/yolov3/data/custom/test/images/*.jpg") + glob.glob(f"{REF}/yolov5/dataset/*/images/*.jpg")):
        h = hashlib.sha256(open(f, "rb").read()).hexdigest()
        if h in seen:
            continue
        seen.add(h)
        shutil.copy(f, os.path.join(OUT, os.path.basename(f)))
    print(len(seen), "files")
