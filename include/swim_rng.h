/*
 * swim_rng.h — the canonical seeded-RNG hook of the lockstep engine (specification constants).
 *
 * The reference draws randomness from ThreadLocalRandom and Collections.shuffle's JVM-global
 * Random (FailureDetectorImpl.java:337,358,372; GossipProtocolImpl.java:329;
 * MembershipProtocolImpl.java:465,469; NetworkEmulator.java:351,364) and has no seed hook.  The
 * engine replaces every draw site with one counter-based Philox4x32-10 block:
 *
 *   word = Philox4x32_10(ctr = {member, (uint32)tick, (stream << 24) | sub24, sub32},
 *                        key = {seed & 0xffffffff, seed >> 32})[0]
 *   nextInt(word, bound) = (uint64)word * bound >> 32
 *   lost(pct, word)      = pct > 0 && (pct >= 100 || nextInt(word, 100) < pct)
 *
 * Both the GPU engine and the CPU oracle implement this independently; the stream ids and the
 * (member, sub24, sub32) key of every draw site are part of the semantics.
 */
#ifndef SWIM_RNG_H
#define SWIM_RNG_H

/* initial state */
#define SWIM_STREAM_INIT_PING 1        /* shuffle of the initial ping list, sub32 = i        */
#define SWIM_STREAM_INIT_REMOTE 2      /* shuffle of the initial gossip remote list          */
#define SWIM_STREAM_INIT_SYNC_PHASE 3  /* periodic-SYNC phase offset when sync_stagger = 1  */
#define SWIM_STREAM_INIT_FD_PHASE 4    /* ping-timer phase offset when timer_stagger = 1    */
#define SWIM_STREAM_INIT_GOSSIP_PHASE 5/* gossip-timer phase offset when timer_stagger = 1  */
/* failure detector (issuer-keyed: member = issuer) */
#define SWIM_STREAM_FD_SHUFFLE 10      /* Collections.shuffle(pingMembers), sub32 = i         */
#define SWIM_STREAM_PING_OUT 11        /* PING issuer -> target outbound loss                 */
#define SWIM_STREAM_ACK_OUT 12         /* PING_ACK target -> issuer outbound loss             */
#define SWIM_STREAM_RELAY_SELECT 13    /* selectPingReqMembers, sub24 = i                     */
#define SWIM_STREAM_PINGREQ_OUT 14     /* PING_REQ issuer -> relay j, sub24 = j               */
#define SWIM_STREAM_TRANSIT_PING_OUT 15/* transit PING relay j -> target                      */
#define SWIM_STREAM_TRANSIT_ACK_OUT 16 /* transit PING_ACK target -> relay j                  */
#define SWIM_STREAM_RELAY_ACK_OUT 17   /* PING_ACK relay j -> issuer                          */
/* message delays (swim_delay.h: u53 from words 0 and 1 of the block), member = the issuer */
#define SWIM_STREAM_PING_DELAY 18      /* PING issuer -> target                               */
#define SWIM_STREAM_ACK_DELAY 19       /* PING_ACK target -> issuer                           */
#define SWIM_STREAM_PINGREQ_DELAY 24   /* PING_REQ issuer -> relay j, sub24 = j               */
#define SWIM_STREAM_TRANSIT_PING_DELAY 25 /* transit PING relay j -> target                   */
#define SWIM_STREAM_TRANSIT_ACK_DELAY 26  /* transit PING_ACK target -> relay j               */
#define SWIM_STREAM_RELAY_ACK_DELAY 27 /* PING_ACK relay j -> issuer                          */
/* gossip (sender-keyed) */
#define SWIM_STREAM_GOSSIP_SHUFFLE 20  /* Collections.shuffle(remoteMembers), sub32 = i       */
#define SWIM_STREAM_GOSSIP_OUT 21      /* GOSSIP_REQ outbound loss, sub24 = target j, sub32 = slab position */
#define SWIM_STREAM_GOSSIP_DELAY 22    /* GOSSIP_REQ delay, member = sender, same sub keys     */
/* membership */
#define SWIM_STREAM_SYNC_SELECT 30     /* selectSyncAddress, sub24 = 0 / 1, sub32 = attempt   */
#define SWIM_STREAM_SYNC_OUT 31        /* SYNC sender -> receiver, sub24 = sender ordinal     */
#define SWIM_STREAM_SYNCACK_OUT 32     /* SYNC_ACK, member = acker, sub24 = inbox rank        */
#define SWIM_STREAM_SYNC_DELAY 33      /* SYNC delay, member = sender, sub24 = sender ordinal */
#define SWIM_STREAM_SYNCACK_DELAY 34   /* SYNC_ACK delay, member = acker, sub24 = inbox rank  */
#define SWIM_STREAM_FETCH_REQ 40       /* GET_METADATA_REQ, sub24 = phase, sub32 = fetch ordinal */
#define SWIM_STREAM_FETCH_RESP 41      /* GET_METADATA_RESP                                   */
#define SWIM_STREAM_FETCH_REQ_DELAY 42 /* GET_METADATA_REQ delay, same sub keys as FETCH_REQ */
#define SWIM_STREAM_FETCH_RESP_DELAY 43 /* GET_METADATA_RESP delay                           */
#define SWIM_STREAM_PING_INSERT 50     /* pingMembers.add(nextInt(size)), sub24 = phase, sub32 = event minor */

#define SWIM_SYNC_SELECT_ATTEMPTS 64

#endif
