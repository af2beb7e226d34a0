"""CIFAR-10 convnet (BASELINE config 3): Caffe cifar10_quick (3x conv 5x5 32/32/64 + pools) -> 64 -> 10, MeanDispNormalizer on uint8 input.

``python -m veles_amd samples/cifar_conv.py -`` (1 GPU), ``... --gpus 0-7``
(8 ranks, one per MI355X).  Synthetic data of the dataset's shape and
random-init weights: the reference sample workflows lived in the absent
Znicz submodule."""
from veles_amd.models import StandardWorkflow
from veles_amd.utils.config import root, fix_contents
import veles_amd.loader  # noqa: F401


def run(load, main):
    cfg = fix_contents(root.cifar_conv)
    load(StandardWorkflow, loader_name=cfg["loader_name"],
         loader_config=cfg["loader"], layers=cfg["layers"],
         decision_config=cfg["decision"],
         snapshotter_config=cfg.get("snapshotter"))
    main()
