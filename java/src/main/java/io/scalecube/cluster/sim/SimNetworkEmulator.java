package io.scalecube.cluster.sim;

import static io.scalecube.cluster.sim.SwimNative.call;

/**
 * NetworkEmulator (cluster-testlib NetworkEmulator.java:59-289) of one simulated member's transport:
 * outbound loss / delay (OutboundSettings, tryFailOutbound :167-181, tryDelayOutbound :190-202 with
 * evaluateDelay :359-369) and inbound pass / block (InboundSettings :212-289), applied by the engine
 * to every message this member sends or receives.
 *
 * <p>Each method replaces a whole OutboundSettings / InboundSettings object as the reference does:
 * loss and delay of a link are set (or removed) together, and the "all" variants first drop every
 * per-link override this member holds ({@code outboundSettings.clear()} / {@code inboundSettings.clear()}).
 * The engine keeps per-link overrides itself; the cluster remembers which links this member set so
 * that a clear can remove them (swimgpu/cluster.py NetworkEmulator issues the same call sequence,
 * tests/test_java_shim.py checks that method by method).  A setting the engine refuses changes nothing:
 * the loss percentage is range-checked before any call and the delay (which the engine may refuse:
 * a mean above its tick cap) is set first, so a refusal leaves loss and delay as they were.
 */
public final class SimNetworkEmulator {
  private final SimulatedCluster cluster;
  private final int member;

  SimNetworkEmulator(SimulatedCluster cluster, int member) {
    this.cluster = cluster;
    this.member = member;
  }

  /** outboundSettings(destination, lossPercent, meanDelay) (:70-74). */
  public void outboundSettings(int destination, int lossPercent, int meanDelay) {
    cluster.run(() -> {
      cluster.checkLossPercent(lossPercent);
      call(SwimNative.SET_LINK_DELAY, "swim_set_link_delay", cluster.engine(), member, destination, meanDelay);
      cluster.noteOutLink(member, destination);
      call(SwimNative.SET_LINK_LOSS, "swim_set_link_loss", cluster.engine(), member, destination, lossPercent);
    });
  }

  /** setDefaultOutboundSettings(lossPercent, meanDelay) (:82-85). */
  public void setDefaultOutboundSettings(int lossPercent, int meanDelay) {
    cluster.run(() -> {
      cluster.checkLossPercent(lossPercent);
      call(SwimNative.SET_DEFAULT_DELAY, "swim_set_default_delay", cluster.engine(), member, meanDelay);
      call(SwimNative.SET_DEFAULT_LOSS, "swim_set_default_loss", cluster.engine(), member, lossPercent);
    });
  }

  /** blockAllOutbound (:88-92): outboundSettings.clear(), then default (100 %, 0 ms). */
  public void blockAllOutbound() {
    cluster.run(() -> {
      for (int d : cluster.takeOutLinks(member)) {
        call(SwimNative.SET_LINK_LOSS, "swim_set_link_loss", cluster.engine(), member, d, -1);
        call(SwimNative.SET_LINK_DELAY, "swim_set_link_delay", cluster.engine(), member, d, -1);
      }
      call(SwimNative.SET_DEFAULT_LOSS, "swim_set_default_loss", cluster.engine(), member, 100);
      call(SwimNative.SET_DEFAULT_DELAY, "swim_set_default_delay", cluster.engine(), member, 0);
    });
  }

  /** unblockAllOutbound (:95-99): outboundSettings.clear(), then default (0 %, 0 ms). */
  public void unblockAllOutbound() {
    cluster.run(() -> {
      for (int d : cluster.takeOutLinks(member)) {
        call(SwimNative.SET_LINK_LOSS, "swim_set_link_loss", cluster.engine(), member, d, -1);
        call(SwimNative.SET_LINK_DELAY, "swim_set_link_delay", cluster.engine(), member, d, -1);
      }
      call(SwimNative.SET_DEFAULT_LOSS, "swim_set_default_loss", cluster.engine(), member, 0);
      call(SwimNative.SET_DEFAULT_DELAY, "swim_set_default_delay", cluster.engine(), member, 0);
    });
  }

  /** blockOutbound(destinations) (:106-120): outboundSettings.put(d, (100 %, 0 ms)). */
  public void blockOutbound(int... destinations) {
    cluster.run(() -> {
      for (int d : destinations) {
        cluster.noteOutLink(member, d);
        call(SwimNative.SET_LINK_LOSS, "swim_set_link_loss", cluster.engine(), member, d, 100);
        call(SwimNative.SET_LINK_DELAY, "swim_set_link_delay", cluster.engine(), member, d, 0);
      }
    });
  }

  /** unblockOutbound(destinations) (:127-139): outboundSettings.remove(d), loss and delay together. */
  public void unblockOutbound(int... destinations) {
    cluster.run(() -> {
      for (int d : destinations) {
        call(SwimNative.SET_LINK_LOSS, "swim_set_link_loss", cluster.engine(), member, d, -1);
        call(SwimNative.SET_LINK_DELAY, "swim_set_link_delay", cluster.engine(), member, d, -1);
      }
    });
  }

  /** inboundSettings(source, shallPass) (:221-225). */
  public void inboundSettings(int source, boolean shallPass) {
    cluster.run(() -> {
      cluster.noteInLink(member, source);
      call(SwimNative.SET_LINK_INBOUND, "swim_set_link_inbound", cluster.engine(), member, source, shallPass ? 1 : 0);
    });
  }

  /** setDefaultInboundSettings(shallPass) (:232-235). */
  public void setDefaultInboundSettings(boolean shallPass) {
    cluster.run(() -> {
      call(SwimNative.SET_DEFAULT_INBOUND, "swim_set_default_inbound", cluster.engine(), member, shallPass ? 1 : 0);
    });
  }

  /** blockAllInbound (:238-242): inboundSettings.clear(), then default shallPass = false. */
  public void blockAllInbound() {
    cluster.run(() -> {
      for (int s : cluster.takeInLinks(member)) {
        call(SwimNative.SET_LINK_INBOUND, "swim_set_link_inbound", cluster.engine(), member, s, -1);
      }
      call(SwimNative.SET_DEFAULT_INBOUND, "swim_set_default_inbound", cluster.engine(), member, 0);
    });
  }

  /** unblockAllInbound (:245-249): inboundSettings.clear(), then default shallPass = true. */
  public void unblockAllInbound() {
    cluster.run(() -> {
      for (int s : cluster.takeInLinks(member)) {
        call(SwimNative.SET_LINK_INBOUND, "swim_set_link_inbound", cluster.engine(), member, s, -1);
      }
      call(SwimNative.SET_DEFAULT_INBOUND, "swim_set_default_inbound", cluster.engine(), member, 1);
    });
  }

  /** blockInbound(sources) (:256-270): inboundSettings.put(s, shallPass = false). */
  public void blockInbound(int... sources) {
    cluster.run(() -> {
      for (int s : sources) {
        cluster.noteInLink(member, s);
        call(SwimNative.SET_LINK_INBOUND, "swim_set_link_inbound", cluster.engine(), member, s, 0);
      }
    });
  }

  /** unblockInbound(sources) (:277-289): inboundSettings.remove(s). */
  public void unblockInbound(int... sources) {
    cluster.run(() -> {
      for (int s : sources) {
        call(SwimNative.SET_LINK_INBOUND, "swim_set_link_inbound", cluster.engine(), member, s, -1);
      }
    });
  }
}
