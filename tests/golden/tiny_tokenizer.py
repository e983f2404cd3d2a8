"""A tiny Qwen2-style byte-level BPE tokenizer for processor fixtures (test
infrastructure only).  The real Qwen2.5 vocabulary files are not available
offline (SURVEY.md §8c "Text tokenizer parity"), so the processor's prompt
layout is pinned with this stand-in: same pre-tokenizer / decoder family and
the same special-token names as Qwen2.5 (<|endoftext|> ... <|video_pad|>), a
small vocabulary trained deterministically on a fixed corpus.

    python tests/golden/tiny_tokenizer.py      # (re)writes tests/golden/tiny_qwen_tokenizer/
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
DIR = os.path.join(HERE, "tiny_qwen_tokenizer")
SPECIALS = ["<|endoftext|>", "<|im_start|>", "<|im_end|>", "<|object_ref_start|>", "<|object_ref_end|>",
            "<|box_start|>", "<|box_end|>", "<|quad_start|>", "<|quad_end|>", "<|vision_start|>", "<|vision_end|>",
            "<|vision_pad|>", "<|image_pad|>", "<|video_pad|>"]
# the Qwen2 pre-tokenization pattern (digits split one by one, letters with one
# leading non-letter, punctuation runs, newline runs)
QWEN2_SPLIT = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*|"
               r"\s*[\r\n]+|\s+(?!\S)|\s+")
CORPUS = [
    " Transform the text provided by various speakers into speech output, utilizing the distinct voice of each "
    "respective speaker.\n",
    " Voice input:\n", " Text input:\n", " Speech output:\n", " Speaker 0:", " Speaker 1:", " Speaker 2:",
    " Speaker 3:", "\n",
    " Hello there, welcome to the show. Today we talk about podcasts and voices.",
    " It's great to be here! How are you doing? Fine, thanks.",
]


def build(path=DIR):
    from tokenizers import Regex, Tokenizer, decoders, models, normalizers, pre_tokenizers, trainers
    from transformers import PreTrainedTokenizerFast
    tok = Tokenizer(models.BPE())
    tok.normalizer = normalizers.NFC()
    tok.pre_tokenizer = pre_tokenizers.Sequence([     # Qwen2's: regex split, then byte-level
        pre_tokenizers.Split(Regex(QWEN2_SPLIT), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=600, special_tokens=SPECIALS, show_progress=False,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(CORPUS * 20, trainer)
    fast = PreTrainedTokenizerFast(tokenizer_object=tok, eos_token="<|endoftext|>", pad_token="<|endoftext|>",
                                   unk_token="<|endoftext|>")
    os.makedirs(path, exist_ok=True)
    fast.save_pretrained(path)
    return path


if __name__ == "__main__":
    print(build())
