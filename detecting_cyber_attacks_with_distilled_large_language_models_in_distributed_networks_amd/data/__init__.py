"""Data layer: synthetic CICIDS2017 generator, featuriser, WordPiece tokenizer, datasets."""
from .dataset import CICIDS2017Dataset, ClientData, DeviceLoader, PackedTokens, build_client_data, short_batch  # noqa: F401
from .featurize import features_to_text, preprocess_data, render_texts, split_60_20_20  # noqa: F401
from .synthetic import CICIDS2017_COLUMNS, generate_cicids2017, write_csv  # noqa: F401
from .tokenizer import DistilBertTokenizer, WordPieceTokenizer  # noqa: F401
