"""Data layer: loader state machine, full-batch device loaders, synthetic
datasets, file / image / pickle / HDF5 / interactive / RESTful loaders."""
from veles_amd.loader.base import (  # noqa: F401
    Loader, LoaderMSE, LoaderMSEMixin, LoaderWithValidationRatio, ILoader,
    UserLoaderRegistry, TEST, VALID, TRAIN, CLASS_NAME)
from veles_amd.loader.fullbatch import (  # noqa: F401
    FullBatchLoader, FullBatchLoaderMSE)
from veles_amd.loader.synthetic import (  # noqa: F401
    SyntheticImageLoader, SyntheticMSELoader)
from veles_amd.loader.image import (  # noqa: F401
    ImageLoader, FileImageLoader, AutoLabelFileImageLoader,
    FileListImageLoader, FullBatchFileImageLoader,
    FullBatchAutoLabelFileImageLoader, FullBatchFileListImageLoader,
    FullBatchImageLoaderMSE)
from veles_amd.loader.pickles import PicklesImageFullBatchLoader  # noqa
from veles_amd.loader.ensemble import EnsembleLoader  # noqa: F401
from veles_amd.loader.loader_hdf5 import FullBatchHDF5Loader  # noqa: F401
from veles_amd.loader.interactive import (  # noqa: F401
    InteractiveLoader, RestfulLoader)
from veles_amd.loader.saver import (  # noqa: F401
    MinibatchesSaver, MinibatchesLoader)
from veles_amd.loader.audio import (  # noqa: F401
    FullBatchAudioLoader, TextLinesLoader, decode_audio)
from veles_amd.loader.queue_loader import (  # noqa: F401
    QueueLoader, QueueLoaderClient)
