package io.scalecube.cluster.gossip;

import io.scalecube.cluster.sim.SimulatedCluster;
import io.scalecube.cluster.transport.api.Message;
import reactor.core.publisher.Flux;
import reactor.core.publisher.Mono;

/**
 * GossipProtocol (GossipProtocol.java:12-29) of one simulated member. spread() hands the message to
 * the engine under a 32-bit handle (swim_spread); the engine runs selectGossipMembers, the spread
 * window, the sweep and the SequenceIdCollector dedupe (GossipProtocolImpl.java:141-368) on the GPU,
 * reports each first receipt as SWIM_EV_GOSSIP (listen(), :209) and the originator's completion after
 * periodsToSpread rounds as SWIM_EV_SPREAD_DONE (the returned Mono, :167-180).
 */
public final class SimGossipProtocol implements GossipProtocol {
  private final SimulatedCluster cluster;
  private final int member;

  public SimGossipProtocol(SimulatedCluster cluster, int member) {
    this.cluster = cluster;
    this.member = member;
  }

  @Override
  public void start() {}

  @Override
  public void stop() {
    cluster.stop(member);
  }

  @Override
  public Mono<String> spread(Message message) {
    return cluster.spread(member, message);
  }

  @Override
  public Flux<Message> listen() {
    return cluster.gossipMessages(member).onBackpressureBuffer();
  }
}
