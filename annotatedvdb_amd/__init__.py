"""annotatedvdb_amd — MI355X-native (gfx950) AnnotatedVDB bin/key path.

Drop-in for the reference's batch variant -> genomic-bin path
(``BinIndex/lib/python/bin_index.py``) and the loader record-prep stage
(``Util/lib/python/loaders/vcf_variant_loader.py:234-348``): end inference,
smallest-enclosing-bin assignment, primary keys and in-batch dedup, computed by
hand-written HIP kernels in ``libavdb_hip.so`` (C ABI: ``include/avdb.h``).

Submodules import torch/the native library lazily so that the host-only parts
(chromosome tables, shard planner, VCF text handling) work without a GPU.
"""

__version__ = "0.1.0"

from .chromosomes import CHROM_NAMES, GRCH38_LENGTHS, chrom_code  # noqa: F401
