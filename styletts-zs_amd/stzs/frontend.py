"""Front ends hosted by PyTorch (SURVEY.md §1 layer L3, out of HIP scope in round 1, §8(f) rank 1).

* `tokenize`: deterministic 178-symbol table (StyleTTS2-family convention: pad, punctuation,
  Latin letters, IPA letters), unknown characters dropped.
* `log_mel`: 24 kHz, 80 mel bins, n_fft 2048, win 1200, hop 300 (SURVEY §8 spec table); an
  in-repo HTK triangular filterbank since torchaudio/librosa are absent in this image.
* `counter_normal`: the counter-based Gaussian used for the harmonic-source noise.  It is a pure
  function of (seed, stream, index) so the HIP source kernel and the CPU oracle draw identical
  noise without moving a [B, 9, 120000] tensor over PCIe.
"""
from __future__ import annotations

import math

import numpy as np
import torch

_PAD = "$"
_PUNCT = ';:,.!?¡¿—…"«»“” '
_LETTERS = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz"
_IPA = ("ɑɐɒæɓʙβɔɕçɗɖðʤəɘɚɛɜɝɞɟʄɡɠɢʛɦɧħɥʜɨɪʝɭɬɫɮʟɱɯɰŋɳɲɴøɵɸθœɶʘɹɺɾɻʀʁɽʂʃʈʧʉʊʋⱱʌɣɤʍχʎʏʑʐʒʔʡʕʢ"
        "ǀǁǂǃˈˌːˑʼʴʰʱʲʷˠˤ˞↓↑→↗↘'̩'ᵻ")


def symbol_table(n_symbols: int = 178) -> list:
    syms = []
    for ch in _PAD + _PUNCT + _LETTERS + _IPA:
        if ch not in syms:
            syms.append(ch)
    i = 0
    while len(syms) < n_symbols:  # reserve slots up to the pinned table size
        syms.append(f"<r{i}>")
        i += 1
    return syms[:n_symbols]


def tokenize(text: str, n_symbols: int = 178) -> list:
    table = {s: i for i, s in enumerate(symbol_table(n_symbols))}
    return [table[c] for c in text if c in table and table[c] != 0]


def mel_filterbank(n_mels: int, n_fft: int, sr: int, fmin: float = 0.0, fmax: float = None) -> torch.Tensor:
    fmax = sr / 2 if fmax is None else fmax
    hz2mel = lambda f: 2595.0 * np.log10(1.0 + f / 700.0)
    mel2hz = lambda m: 700.0 * (10 ** (m / 2595.0) - 1.0)
    mpts = np.linspace(hz2mel(fmin), hz2mel(fmax), n_mels + 2)
    fpts = mel2hz(mpts)
    freqs = np.linspace(0, sr / 2, n_fft // 2 + 1)
    fb = np.zeros((n_mels, n_fft // 2 + 1))
    for m in range(n_mels):
        lo, ce, hi = fpts[m], fpts[m + 1], fpts[m + 2]
        up = (freqs - lo) / max(ce - lo, 1e-9)
        dn = (hi - freqs) / max(hi - ce, 1e-9)
        fb[m] = np.maximum(0.0, np.minimum(up, dn))
    return torch.from_numpy(fb).float()


def log_mel(wav: torch.Tensor, spec, fb: torch.Tensor = None) -> torch.Tensor:
    """wav [B, N] fp32 -> log-mel [B, n_mels, frames] (device of `wav`)."""
    if fb is None:
        fb = mel_filterbank(spec.n_mels, spec.mel_nfft, spec.sr)
    fb = fb.to(wav.device)
    win = torch.hann_window(spec.mel_win, device=wav.device)
    X = torch.stft(wav, spec.mel_nfft, hop_length=spec.hop, win_length=spec.mel_win,
                   window=win, center=True, return_complex=True)
    power = X.real ** 2 + X.imag ** 2
    mel = torch.matmul(fb, power)
    return torch.log(torch.clamp(mel, min=1e-5))


# ---- counter-based RNG (lowbias32 hash + Box-Muller), mirrored bit-for-bit in csrc/source.hip ----
_M1 = np.uint32(0x7FEB352D)
_M2 = np.uint32(0x846CA68B)


def hash32(x):
    x = np.asarray(x, dtype=np.uint32)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint32(16))
        x = x * _M1
        x = x ^ (x >> np.uint32(15))
        x = x * _M2
        x = x ^ (x >> np.uint32(16))
    return x


def stream_key(seed: int, stream: int) -> np.uint32:
    with np.errstate(over="ignore"):
        s1 = hash32(np.uint32(seed & 0xFFFFFFFF) + np.uint32(0x9E3779B9))
        return hash32(s1 ^ np.uint32(stream & 0xFFFFFFFF))


def counter_uniform_pair(key, idx):
    """(u1 in (0,1], u2 in [0,1)) as float64 from 24-bit hashes of counters 2*idx, 2*idx+1."""
    idx = np.asarray(idx, dtype=np.uint32)
    with np.errstate(over="ignore"):
        a = hash32(key ^ hash32(idx * np.uint32(2)))
        b = hash32(key ^ hash32(idx * np.uint32(2) + np.uint32(1)))
    u1 = ((a >> np.uint32(8)).astype(np.float64) + 1.0) * (1.0 / 16777216.0)
    u2 = (b >> np.uint32(8)).astype(np.float64) * (1.0 / 16777216.0)
    return u1, u2


def counter_normal(key, idx) -> np.ndarray:
    u1, u2 = counter_uniform_pair(key, idx)
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)).astype(np.float32)


def initial_phase(key) -> np.float32:
    """random initial phase of a harmonic stream, uniform [0,1) from the counter 0xFFFFFFFF"""
    with np.errstate(over="ignore"):
        a = hash32(key ^ np.uint32(0xA5A5A5A5))
    return np.float32((a >> np.uint32(8)).astype(np.float64) * (1.0 / 16777216.0))
