"""Loss collector with the reference interface (lib/loss.py:8-51, pggan/loss.py:4-27).

The losses are computed on the GPU by the step engine (`pg_bce_loss`,
`pg_r1_penalty`) into a device buffer; `loss_dict` is filled lazily (one device
sync, only when read) with the same keys and 4-decimal rounding as the reference
(`pggan/loss.py:12,23-25`), so the hot loop has no `.item()` syncs.
"""
import time


class LossInterface:
    """lib/loss.py:8-51."""

    def __init__(self, args):
        self.args = args
        self.start_time = time.time()
        self._loss_dict = {}
        self._buf = None
        self._mode = "r1"

    def attach(self, buf, mode="r1"):
        self._buf = buf
        self._mode = mode

    @property
    def loss_dict(self):
        if self._buf is not None:
            v = self._buf.detach().float().cpu().tolist()
            L_real, L_fake, reg, L_G, drift = v[0], v[1], v[2], v[3], v[4]
            self._loss_dict.update({
                "L_D_real": round(L_real, 4), "L_D_fake": round(L_fake, 4),
                "L_D": round(L_real + L_fake + reg + drift, 4), "L_G": round(L_G, 4)})
            if self._mode != "r1":
                # key names of the reference's commented-out WGAN-GP collector (pggan/loss.py:46-50)
                self._loss_dict["L_D_gp"] = round(reg, 4)
                self._loss_dict["L_D_eps"] = round(drift, 4)
            self._buf = None
        return self._loss_dict

    def print_loss(self, global_step):
        """lib/loss.py:23-31."""
        seconds = int(time.time() - self.start_time)
        d = self.loss_dict
        print("")
        print(f"[ {seconds//3600//24:02}d {(seconds//3600)%24:02}h {(seconds//60)%60:02}m "
              f"{seconds%60:02}s ]")
        print(f"steps: {global_step:06} / {self.args.max_step}")
        print(f'lossD: {d["L_D"]} | lossG: {d["L_G"]}')


class WGANGPLoss(LossInterface):
    """pggan/loss.py:4-100: L_D = BCE(real,1) + BCE(fake,0) + R1 (live path);
    L_G = W_adv * BCE(fake,1).  gp_mode="wgan-gp" switches the regulariser to the
    (dead in the reference) interpolate->D->grad-norm penalty of :54-92 plus the drift
    term W_drift_D * sum D(real)^2 of :94-100, both differentiated into D's gradient."""
