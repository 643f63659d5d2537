package io.scalecube.cluster.fdetector;

import io.scalecube.cluster.Member;
import io.scalecube.cluster.membership.MemberStatus;
import io.scalecube.cluster.sim.SimulatedCluster;
import reactor.core.publisher.Flux;

/**
 * FailureDetector (FailureDetector.java:12-25) of one simulated member: its doPing / ping-req /
 * DEST_GONE results (FailureDetectorImpl.java:126-404) are computed by the engine's k_fd kernel and
 * arrive here as the SWIM_EV_FD_* events of this viewer. Lives in the reference's package because
 * FailureDetectorEvent's constructor is package-private (FailureDetectorEvent.java:12-15).
 */
public final class SimFailureDetector implements FailureDetector {
  private final SimulatedCluster cluster;
  private final int member;

  public SimFailureDetector(SimulatedCluster cluster, int member) {
    this.cluster = cluster;
    this.member = member;
  }

  public static FailureDetectorEvent event(Member m, MemberStatus status) {
    return new FailureDetectorEvent(m, status);
  }

  /** The detector runs from the member's start on (the engine's FD timer, FailureDetectorImpl.java:102-106). */
  @Override
  public void start() {}

  /** FailureDetectorImpl.stop: the member's transport stops with it. */
  @Override
  public void stop() {
    cluster.stop(member);
  }

  @Override
  public Flux<FailureDetectorEvent> listen() {
    return cluster.failureDetectorEvents(member).onBackpressureBuffer();
  }
}
