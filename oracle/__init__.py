"""CPU oracle for the per-frame alpha-matting path — TEST INFRASTRUCTURE ONLY.

This package is a plain-numpy restatement of the reference's hot path
(tangih/video-matting: unet.py, unet_simple.py, small.py, refine.py, flow.py,
reader.read_flow, the train.py loss).  It exists to CHECK the HIP path:

* only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
  ``cpu_baseline`` leg may import it;
* the product path (``video-matting_amd/``) never imports, links or executes
  anything under ``oracle/`` — it fails loudly when its HIP library is missing.

Pinning: the reference is TensorFlow-1.x + OpenCV, both
absent from this image.  ``tests/golden/make_golden.py`` runs the reference's
OWN graph-builder / flow / reader / loss code (imported from /root/reference)
on top of a literal TF/cv2 op shim and commits the outputs as fixtures; the
oracle here is checked against those fixtures.  That pins wiring, channel and
concat orders, filter construction, RNG draw order, BN/ReLU/bias placement and
``correct_alpha``/``read_flow`` bit-exactly (those run for real); the TF/OpenCV
op semantics themselves (Appendix A of SURVEY.md) are restated from library
documentation and are therefore "parity unpinned" against real TF/OpenCV.
"""

from . import ops, models, flow  # noqa: F401
