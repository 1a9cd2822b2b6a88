"""Models: arena-backed DistilBERT ``DDoSClassifier`` (+ BERT-base teacher for distillation)."""
from .arena import ParamArena  # noqa: F401
from .distilbert import DDoSClassifier, DistilBertConfig, reference_state_dict_keys  # noqa: F401
from .bert import BertTeacherClassifier, bert_base_config, kd_loss  # noqa: F401
