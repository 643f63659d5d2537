package io.scalecube.cluster.membership;

import io.scalecube.cluster.Member;
import io.scalecube.cluster.sim.SimulatedCluster;
import io.scalecube.cluster.sim.SwimNative;
import io.scalecube.net.Address;
import java.util.ArrayList;
import java.util.Collection;
import java.util.List;
import java.util.Map;
import java.util.Optional;
import java.util.TreeMap;
import reactor.core.publisher.Flux;
import reactor.core.publisher.Mono;

/**
 * MembershipProtocol (MembershipProtocol.java:14-65) of one simulated member: its membership table
 * is row `member` of the engine's view matrix (swim_read_view), its events the engine's ADDED /
 * REMOVED / LEAVING / UPDATED events of this viewer, in the engine's canonical order.
 */
public final class SimMembershipProtocol implements MembershipProtocol {
  private final SimulatedCluster cluster;
  private final int member;

  public SimMembershipProtocol(SimulatedCluster cluster, int member) {
    this.cluster = cluster;
    this.member = member;
  }

  /** A member of the converged start runs already; a free slot starts through its seeds (start0 :250-291). */
  @Override
  public Mono<Void> start() {
    return Mono.fromRunnable(() -> {
      if (!SwimNative.cellInTable(cluster.view(member)[member])) cluster.start(member);
    });
  }

  @Override
  public void stop() {
    cluster.stop(member);
  }

  @Override
  public Flux<MembershipEvent> listen() {
    return cluster.membershipEvents(member).onBackpressureBuffer();
  }

  /** members() (:313-315): subjects in `members` (ADDED and not REMOVED). */
  @Override
  public Collection<Member> members() {
    long[] row = cluster.view(member);
    List<Member> out = new ArrayList<>();
    for (int s = 0; s < row.length; s++) if (SwimNative.cellInMembers(row[s])) out.add(cluster.member(s));
    return out;
  }

  @Override
  public Collection<Member> otherMembers() {
    Collection<Member> all = members();
    all.removeIf(m -> m.id().equals(member().id()));
    return all;
  }

  @Override
  public Member member() {
    return cluster.member(member);
  }

  @Override
  public Optional<Member> member(String id) {
    int s = cluster.slotOf(id);
    return s >= 0 && s < cluster.capacity() && SwimNative.cellInMembers(cluster.view(member)[s])
        ? Optional.of(cluster.member(s)) : Optional.empty();
  }

  @Override
  public Optional<Member> member(Address address) {
    return members().stream().filter(m -> m.address().equals(address)).findFirst();
  }

  /** getMembershipRecords (:903-905), package-private in the reference too (the tests read it). */
  Map<String, MembershipRecord> getMembershipRecords() {
    long[] row = cluster.view(member);
    Map<String, MembershipRecord> out = new TreeMap<>();
    for (int s = 0; s < row.length; s++) {
      if (!SwimNative.cellInTable(row[s])) continue;
      MemberStatus st = MemberStatus.values()[SwimNative.cellStatus(row[s])];
      out.put(cluster.member(s).id(), new MembershipRecord(cluster.member(s), st, SwimNative.cellInc(row[s])));
    }
    return out;
  }
}
