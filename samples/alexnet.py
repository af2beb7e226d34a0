"""AlexNet-ImageNet (BASELINE config 4, the headline benchmark): one-tower Caffe AlexNet 227x227, synchronous data parallel over RCCL with --gpus 0-7.

``python -m veles_amd samples/alexnet.py -`` (1 GPU), ``... --gpus 0-7``
(8 ranks, one per MI355X).  Synthetic data of the dataset's shape and
random-init weights: the reference sample workflows lived in the absent
Znicz submodule."""
from veles_amd.models import StandardWorkflow
from veles_amd.utils.config import root, fix_contents
import veles_amd.loader  # noqa: F401


def run(load, main):
    cfg = fix_contents(root.alexnet)
    load(StandardWorkflow, loader_name=cfg["loader_name"],
         loader_config=cfg["loader"], layers=cfg["layers"],
         decision_config=cfg["decision"],
         snapshotter_config=cfg.get("snapshotter"))
    main()
