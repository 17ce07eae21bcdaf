"""CPU oracle for the segmentation training path -- TEST INFRASTRUCTURE ONLY.

This package is a CPU restatement (torch-CPU, float64 by default) of the
TensorFlow 1.x semantics that the reference's hot path relies on
(`Network/model/FCN.py`, `Network/utils/utils.py`, `Network/model/FCDenseNet.py`).
It exists to *check* the MI355X HIP path, never to run it:

* only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline`
  leg may import it;
* the product package (`semanticsegmentation_tensorflow_amd`) never imports
  it and has no CPU fallback -- it fails loudly without its HIP library.

Parity pinning status
---------------------
The reference ships no tests, fixtures or golden vectors, and its arithmetic
lives in TensorFlow 1.x kernels that are not installed here.
**Parity is therefore unpinned by the reference itself.**  What pins this
oracle instead:

1. every op is restated from TF1's documented semantics (SURVEY.md
   Appendix A), each function citing the reference call site it follows;
2. the conv / transposed-conv / pool restatements are cross-checked against
   an independent pure-numpy loop implementation (`oracle/naive.py`);
3. hand-derived known answers for the TF-specific rules (asymmetric SAME
   padding, the conv2d_transpose shape rule, TF1 Adam's epsilon placement,
   max-pool tie routing) are asserted in `tests/test_oracle.py`;
4. golden fixtures generated from this oracle are committed under
   `tests/golden/` together with the script that made them.
"""
