"""VGG-16 ImageNet in fp8 (BASELINE config 5): 13 conv 3x3 + 5 pools + 4096-4096-1000; e4m3 activations/weights and e5m2 gradients on the fp8 MFMA kernels, fp32 master weights.

``python -m veles_amd samples/vgg16.py -`` (1 GPU), ``... --gpus 0-7``
(8 ranks, one per MI355X).  Synthetic data of the dataset's shape and
random-init weights: the reference sample workflows lived in the absent
Znicz submodule."""
from veles_amd.models import StandardWorkflow
from veles_amd.utils.config import root, fix_contents
import veles_amd.loader  # noqa: F401


def run(load, main):
    cfg = fix_contents(root.vgg16)
    load(StandardWorkflow, loader_name=cfg["loader_name"],
         loader_config=cfg["loader"], layers=cfg["layers"],
         decision_config=cfg["decision"],
         snapshotter_config=cfg.get("snapshotter"))
    main()
