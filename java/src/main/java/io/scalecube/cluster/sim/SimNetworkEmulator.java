package io.scalecube.cluster.sim;

import static io.scalecube.cluster.sim.SwimNative.call;

/**
 * NetworkEmulator (cluster-testlib NetworkEmulator.java:59-298) of one simulated member's transport:
 * outbound loss / delay (OutboundSettings, tryFailOutbound :167-181, tryDelayOutbound :190-202 with
 * evaluateDelay :359-369) and inbound pass / block (InboundSettings :212-289), applied by the engine
 * to every message this member sends or receives.
 */
public final class SimNetworkEmulator {
  private final SimulatedCluster cluster;
  private final int member;

  SimNetworkEmulator(SimulatedCluster cluster, int member) {
    this.cluster = cluster;
    this.member = member;
  }

  /** setDefaultOutboundSettings(lossPercent, meanDelay) (:69-83). */
  public void setDefaultOutboundSettings(int lossPercent, int meanDelay) {
    cluster.run(() -> {
      call(SwimNative.SET_DEFAULT_LOSS, "swim_set_default_loss", cluster.engine(), member, lossPercent);
      if (meanDelay > 0) // delays need a single-shard engine (swim.h)
        call(SwimNative.SET_DEFAULT_DELAY, "swim_set_default_delay", cluster.engine(), member, meanDelay);
    });
  }

  /** outboundSettings(destination, lossPercent, meanDelay) (:59-67). */
  public void outboundSettings(int destination, int lossPercent, int meanDelay) {
    cluster.run(() -> {
      call(SwimNative.SET_LINK_LOSS, "swim_set_link_loss", cluster.engine(), member, destination, lossPercent);
      if (meanDelay > 0)
        call(SwimNative.SET_LINK_DELAY, "swim_set_link_delay", cluster.engine(), member, destination, meanDelay);
    });
  }

  /** blockOutbound(destinations) (:115-127): 100 % loss. */
  public void blockOutbound(int... destinations) {
    for (int d : destinations) outboundSettings(d, 100, 0);
  }

  /** unblockOutbound(destinations) (:129-139): back to the default loss (-1 clears the link setting). */
  public void unblockOutbound(int... destinations) {
    cluster.run(() -> {
      for (int d : destinations) call(SwimNative.SET_LINK_LOSS, "swim_set_link_loss", cluster.engine(), member, d, -1);
    });
  }

  /** blockAllOutbound (:141-147). */
  public void blockAllOutbound() {
    cluster.run(() -> call(SwimNative.SET_DEFAULT_LOSS, "swim_set_default_loss", cluster.engine(), member, 100));
  }

  /** inboundSettings(source, shallPass) (:237-247) / blockInbound (:249-261) / unblockInbound (:263-273). */
  public void inboundSettings(int source, boolean shallPass) {
    cluster.run(() -> call(SwimNative.SET_LINK_INBOUND, "swim_set_link_inbound", cluster.engine(), member, source,
        shallPass ? 1 : 0));
  }

  public void blockInbound(int... sources) {
    for (int s : sources) inboundSettings(s, false);
  }

  /** setDefaultInboundSettings(shallPass) (:219-227); blockAllInbound (:275-281). */
  public void setDefaultInboundSettings(boolean shallPass) {
    cluster.run(() -> call(SwimNative.SET_DEFAULT_INBOUND, "swim_set_default_inbound", cluster.engine(), member,
        shallPass ? 1 : 0));
  }
}
