"""HOTPATH spec v0 — the pinned architecture of the StyleTTS-ZS synthesis hot path.

The upstream repository publishes no code (`/root/reference/README.md:15-16`, "Inference /
Under construction"); its only technical content is the abstract (`README.md:5`): text plus
fixed-length time-varying style codes, a style diffusion model with classifier-free guidance,
a distilled few-step sampler.  Every dimension below is therefore a build pin
(SURVEY.md §8 "HOTPATH spec v0"), following StyleTTS/StyleTTS2-family conventions where the
abstract is silent.  Changing any field changes the oracle and the golden fixtures together.

Deviations from the StyleTTS2 family, all recorded in DESIGN.md §2:
  * harmonic-source features are the (real, imag) STFT parts, not (magnitude, atan2 phase):
    atan2 is discontinuous at the branch cut, which would make parity ill-posed;
  * the generator has no `noise_res` blocks (matches SURVEY.md's 185 GF decoder cost model);
  * the denoiser uses adaLN-single (one shared modulation linear + per-layer learned table).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field


@dataclass(frozen=True)
class Spec:
    name: str = "v0"
    # audio framing (SURVEY §8 spec table): 24 kHz, 80 fps mel, 40 fps aligned frames
    sr: int = 24000
    hop: int = 300                 # samples per 80-fps frame
    # text
    n_symbols: int = 178
    d_txt: int = 512
    te_layers: int = 3
    te_kernel: int = 5             # CNN stack, then one BiLSTM d_txt -> 2 x d_txt/2 (StyleTTS2 TextEncoder)
    # style codes: L_s codes x (style_ac + style_pr)
    L_s: int = 50
    style_ac: int = 128
    style_pr: int = 128
    # prompt encoder (front end, hosted)
    n_mels: int = 80
    mel_nfft: int = 2048
    mel_win: int = 1200
    pe_ch: int = 256
    # discrete style codes (README.md:5): product VQ of each prompt code row, code_dim / vq_group groups of
    # vq_group values, one vq_size-entry codebook per group
    vq_group: int = 8
    vq_size: int = 256
    vq_std: float = 0.2            # codebook init scale (~ the prompt projection's output std)
    # denoiser
    dn_d: int = 512
    dn_heads: int = 8
    dn_layers: int = 6
    dn_ffn: int = 2048
    dn_fourier: int = 256
    sigma_data: float = 0.2
    sigma_min: float = 1e-4
    sigma_max: float = 3.0
    rho: float = 9.0
    # predictor
    pr_hid: int = 512              # BiLSTM output width (2 x pr_hid/2)
    pr_layers: int = 3
    dur_bins: int = 50
    f0n_ch: tuple = (512, 256, 256)
    f0_bias: float = 150.0         # F0 head bias init (Hz) so random-init F0 is voiced
    # decoder
    dec_enc: int = 1024
    dec_asr_res: int = 64
    dec_out: int = 512
    gen_ch: tuple = (256, 128)
    up_rates: tuple = (10, 6)
    up_kernels: tuple = (20, 12)
    rb_kernels: tuple = (3, 7, 11)
    rb_dils: tuple = (1, 3, 5)
    n_fft: int = 20
    istft_hop: int = 5
    harmonic_num: int = 8
    sine_amp: float = 0.1
    noise_std: float = 0.003
    voiced_threshold: float = 10.0

    # ---- derived ----
    @property
    def code_dim(self) -> int:
        return self.style_ac + self.style_pr

    @property
    def n_bins(self) -> int:
        return self.n_fft // 2 + 1

    @property
    def har_ch(self) -> int:
        return 2 * self.n_bins

    @property
    def frame40(self) -> int:
        """samples per aligned (duration) frame = 2 mel frames"""
        return 2 * self.hop

    @property
    def dn_head_dim(self) -> int:
        return self.dn_d // self.dn_heads

    @property
    def lstm_h(self) -> int:
        return self.pr_hid // 2

    @property
    def pr_in(self) -> int:
        return self.d_txt + self.style_pr

    def check(self) -> "Spec":
        prod = 1
        for r in self.up_rates:
            prod *= r
        assert prod * self.istft_hop == self.hop, "upsampling x iSTFT hop must equal the mel hop"
        for r, k in zip(self.up_rates, self.up_kernels):
            assert k == 2 * r, "ConvTranspose kernels must be 2x stride (polyphase form)"
        assert self.d_txt == self.pr_hid, "predictor hidden width equals the text width (StyleTTS2)"
        assert self.dn_d % self.dn_heads == 0
        assert self.code_dim % self.vq_group == 0 and self.vq_group in (4, 8, 16)
        assert self.d_txt % 64 == 0 and self.d_txt // 2 <= 256, "text BiLSTM: H % 32 == 0, H <= 256 (csrc/lstm.hip)"
        return self

    def replace(self, **kw) -> "Spec":
        return dataclasses.replace(self, **kw).check()


SPEC_V0 = Spec().check()

# Small-dimension variant with the same topology, for golden fixtures and CPU tests.
SPEC_TINY = Spec(
    name="tiny",
    d_txt=64, L_s=8, style_ac=32, style_pr=32, pe_ch=32, n_mels=16,
    dn_d=64, dn_heads=2, dn_layers=2, dn_ffn=128, dn_fourier=32,
    pr_hid=64, pr_layers=2, dur_bins=8, f0n_ch=(64, 32, 32),
    dec_enc=96, dec_asr_res=16, dec_out=64, gen_ch=(32, 16),
).check()


def sample_count(spec: Spec, n_frames40: int) -> int:
    """waveform length for T40 aligned frames: T80*hop (iSTFT over T80*hop/istft_hop + 1 frames)."""
    return n_frames40 * spec.frame40
